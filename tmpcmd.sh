timeout -k 10 400 python bench.py > gpurun_out/r01_bench.json 2> gpurun_out/r01_bench.err && \
sh ppo.c_amd/tools/pmc_bench.sh r01
