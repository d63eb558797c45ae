for v in base sgb1 sgb2 sgb1all sgb2all; do
  timeout -k 10 120 python ppo.c_amd/tools/gemm_sweep.py --main --lib ppo.c_amd/lib/variants/libppo_$v.so --cfgs 0,4 > gpurun_out/var_$v.log 2>&1 || exit 1
done
