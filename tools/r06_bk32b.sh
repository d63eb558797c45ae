#!/bin/sh
# r06_bk32b.sh TAG — 32-k small tiles for the forwards only (PPO_X3_BK32=nt) vs none (default), alternating, G = 8 shard and C3
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
for i in 1 2; do
  PPO_COMM_SELF=1 timeout -k 10 240 python bench.py --emulate-world 8 --no-cpu-baseline --no-rollout > $O/shard8_$i.log 2>&1 || exit 1
  PPO_COMM_SELF=1 PPO_X3_BK32=nt timeout -k 10 240 python bench.py --emulate-world 8 --no-cpu-baseline --no-rollout > $O/shard8_nt_$i.log 2>&1 || exit 1
  timeout -k 10 240 python bench.py --config c3 --no-cpu-baseline --no-rollout > $O/c3_$i.log 2>&1 || exit 1
  PPO_X3_BK32=nt timeout -k 10 240 python bench.py --config c3 --no-cpu-baseline --no-rollout > $O/c3_nt_$i.log 2>&1 || exit 1
done
