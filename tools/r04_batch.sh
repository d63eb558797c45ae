#!/bin/sh
# r04_batch.sh TAG — cluster tests, the C4 B = 64 phase (stamps + bench), then same-box A/Bs: grad_W
# TN tile (PPO_X3_TN_CFG 3 vs 5) at C4, and the fused head's rows per wave slot at the G = 8 shard
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_cluster.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log; grep "512 .* steps vs oracle" $O/tests.log
sh tools/r04_deep.sh $1 || exit 1
sh tools/ab_env.sh PPO_X3_TN_CFG 3 5 > $O/ab_tn.txt 2>&1 || exit 1
cat $O/ab_tn.txt
PPO_COMM_SELF=1 BENCH_ARGS="--emulate-world 8" sh tools/ab_env.sh PPO_OUTHEAD_RPS 16 4 2 > $O/ab_rps_shard.txt 2>&1 || exit 1
cat $O/ab_rps_shard.txt
