timeout -k 10 200 python ppo.c_amd/tools/gemm_x3_sweep.py --ops=0,1,2 --cfgs=0,7 --shapes="32768,512,512;32768,376,512;8192,512,512" > gpurun_out/x3_pp.txt 2>&1 && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_x3.py -x -q --timeout 120 --timeout-method thread > gpurun_out/x3_pp_test.log 2>&1
