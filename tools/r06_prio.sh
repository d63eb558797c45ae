#!/bin/sh
# r06_prio.sh TAG — stream priorities (PPO_STREAM_PRIO=1: value loop's stream high, policy's low) vs default:
# C3, C4 and the G = 8 shard, interleaved twice
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
for i in 1 2; do for pr in 1 0; do
  PPO_STREAM_PRIO=$pr timeout -k 10 200 python bench.py --config c3 --no-cpu-baseline --no-rollout > $O/c3_p${pr}_$i.log 2>&1 || exit 1
  PPO_STREAM_PRIO=$pr timeout -k 10 240 python bench.py --no-cpu-baseline --no-rollout > $O/c4_p${pr}_$i.log 2>&1 || exit 1
  PPO_STREAM_PRIO=$pr PPO_COMM_SELF=1 timeout -k 10 240 python bench.py --emulate-world 8 --no-cpu-baseline --no-rollout > $O/sh_p${pr}_$i.log 2>&1 || exit 1
done; done
