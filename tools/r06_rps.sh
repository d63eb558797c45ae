#!/bin/sh
# r06_rps.sh TAG — out_head_kernel rows per wave slot (PPO_OUT_HEAD_RPS): C3 and the G = 8 shard at 16 / 8 / 4
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
for i in 1 2; do for r in 16 8 4; do
  PPO_OUT_HEAD_RPS=$r timeout -k 10 200 python bench.py --config c3 --no-cpu-baseline --no-rollout > $O/c3_r${r}_$i.log 2>&1 || exit 1
done; done
