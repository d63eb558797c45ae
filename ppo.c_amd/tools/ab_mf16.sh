#!/bin/bash
# ab_mf16.sh TAG — x3 16×16×32 paired form (PPO_X3_MF16=1) vs the 32×32×16 form: parity tests
# under the paired form, then isolated x3 launch timings and the default bench line for both forms
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit 1;; esac; }
PPO_X3_MF16=1 timeout -k 10 500 python -u -m pytest tests/test_gpu_x3.py tests/test_gpu_gemm_cfgs.py tests/test_gpu_ops.py \
    tests/test_gpu_index.py tests/test_gpu_update.py -x -q --timeout 200 --timeout-method thread > $O/test_mf1.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/test_mf1.log; fatal $rc pytest
for mf in 0 1; do
    PPO_X3_MF16=$mf timeout -k 10 120 python ppo.c_amd/tools/x3_bench.py --iters 30 > $O/x3_mf$mf.log 2>&1 || exit 1
done
for mf in 0 1 0 1; do
    PPO_X3_MF16=$mf timeout -k 10 150 python bench.py --no-cpu-baseline >> $O/bench_mf$mf.log 2>&1 || exit 1
done
