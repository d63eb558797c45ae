#!/bin/sh
# r06_bk32.sh TAG — the -m gpu suite, then the 32-k small tiles A/B (default vs PPO_X3_BK32=0) at the G = 8
# shard and C3, alternating, and the small-shape engine table
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 || exit 1
for i in 1 2; do
  PPO_COMM_SELF=1 timeout -k 10 240 python bench.py --emulate-world 8 --no-cpu-baseline --no-rollout > $O/shard8_$i.log 2>&1 || exit 1
  PPO_COMM_SELF=1 PPO_X3_BK32=0 timeout -k 10 240 python bench.py --emulate-world 8 --no-cpu-baseline --no-rollout > $O/shard8_bk16_$i.log 2>&1 || exit 1
  timeout -k 10 240 python bench.py --config c3 --no-cpu-baseline --no-rollout > $O/c3_$i.log 2>&1 || exit 1
  PPO_X3_BK32=0 timeout -k 10 240 python bench.py --config c3 --no-cpu-baseline --no-rollout > $O/c3_bk16_$i.log 2>&1 || exit 1
done
timeout -k 10 120 python tools/engine_small_shapes.py > $O/engines.log 2>&1 || exit 1
