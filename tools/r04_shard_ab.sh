#!/bin/sh
# r04_shard_ab.sh TAG — same-box A/Bs at the G = 8 shard: grad_W split-K target (workgroups per launch)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
PPO_COMM_SELF=1 BENCH_ARGS="--emulate-world 8" sh tools/ab_env.sh PPO_X3_SPLIT_TARGET 256 128 512 > $O/ab_split_shard.txt 2>&1 || { cat $O/ab_split_shard.txt; exit 1; }
cat $O/ab_split_shard.txt
