#!/bin/bash
# ab_smallm.sh TAG — small-M GEMM kernels (B = 64 minibatch products): parity tests, then a same-box
# A/B of libppo builds at C3 B = 64 (lib/libppo_base.so = the previous build)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_gemm_cfgs.py tests/test_gpu_update.py tests/test_gpu_api.py \
    tests/test_gpu_rollout.py -x -q --timeout 200 --timeout-method thread > $O/test.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/test.log
case $rc in 0) ;; *) exit 1;; esac
BENCH_ARGS="--config c3 --batch 64 --steps 2 --warmup 1" sh tools/ab_lib.sh ppo.c_amd/lib/libppo_base.so ppo.c_amd/lib/libppo.so > $O/ab_c3b64.log 2>&1 || exit 1
