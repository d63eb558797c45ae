#!/bin/sh
# r06_fused.sh TAG — the A = 17 policy output layer in one launch (policy_out_fused_kernel, default) vs the
# forward GEMM + out_bwd_wide_kernel<HEAD> (PPO_POLICY_FUSED=0): the tests that cover them, then C4 and the
# G = 8 shard interleaved twice
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_update.py -x -v -k "wide or graph" --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || exit 1
for i in 1 2; do for f in 1 0; do
  PPO_POLICY_FUSED=$f timeout -k 10 240 python bench.py --no-cpu-baseline --no-rollout > $O/c4_f${f}_$i.log 2>&1 || exit 1
done; done
for f in 1 0; do
  PPO_POLICY_FUSED=$f PPO_COMM_SELF=1 timeout -k 10 240 python bench.py --emulate-world 8 --no-cpu-baseline --no-rollout > $O/shard_f${f}.log 2>&1 || exit 1
done
