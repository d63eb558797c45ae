#!/bin/sh
# r06_wide.sh TAG — the wide output-layer backward with its next rows' x in flight (libppo) vs issued after
# each block's stores (variant widenopf): the tests that cover it, then C4 interleaved twice
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_update.py tests/test_gpu_gemm_cfgs.py tests/test_gpu_production.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 240 python bench.py --no-cpu-baseline --no-rollout > $O/c4_$i.log 2>&1 || exit 1
  PPO_LIB=$R/ppo.c_amd/lib/variants/libppo_widenopf.so timeout -k 10 240 python bench.py --no-cpu-baseline --no-rollout > $O/c4_nopf_$i.log 2>&1 || exit 1
done
