#!/bin/sh
# r06_tn.sh TAG — grad_W tile configuration A/B at the small products (G = 8 shard, C3): cfg 3 (default: 128x128,
# two k-groups, 144 KiB) vs cfg 2 (128x128, one k-group, 72 KiB) vs cfg 4 (64x64, 36 KiB); the x3 accuracy
# tests under each
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
for c in 2 4; do
  PPO_X3_TN_CFG=$c timeout -k 10 300 python -u -m pytest tests/test_gpu_x3.py -x -q -s --timeout 200 --timeout-method thread > $O/x3tests_$c.log 2>&1 || exit 1
done
for i in 1 2; do
  for c in 3 2 4; do
    PPO_X3_TN_CFG=$c PPO_COMM_SELF=1 timeout -k 10 240 python bench.py --emulate-world 8 --no-cpu-baseline --no-rollout > $O/shard8_tn${c}_$i.log 2>&1 || exit 1
    PPO_X3_TN_CFG=$c timeout -k 10 240 python bench.py --config c3 --no-cpu-baseline --no-rollout > $O/c3_tn${c}_$i.log 2>&1 || exit 1
  done
done
