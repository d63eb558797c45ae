#!/bin/sh
# final_configs.sh TAG — every config's bench line on one box (C4, the G = 8 shard, C3, C2, C5)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
timeout -k 10 240 python3 bench.py --no-rollout > $O/c4.json 2>&1 || exit 1
PPO_COMM_SELF=1 timeout -k 10 200 python3 bench.py --emulate-world 8 --no-cpu-baseline --no-rollout > $O/shard8.json 2>&1 || exit 1
timeout -k 10 200 python3 bench.py --config c3 --no-rollout > $O/c3.json 2>&1 || exit 1
timeout -k 10 200 python3 bench.py --config c2 --no-rollout > $O/c2.json 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --config c5 --no-cpu-baseline --no-rollout > $O/c5.json 2>&1
