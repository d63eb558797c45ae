#!/bin/sh
# fused heads: fewer workgroups (PPO_OUTHEAD_RPS 32 / 64) vs the default 16 at C3, C5 and the shard
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/rpshi
BENCH_ARGS="--config c3" timeout -k 10 300 sh tools/ab_env.sh PPO_OUTHEAD_RPS 16 32 64 > gpurun_out/rpshi/c3.txt 2>&1 && cat gpurun_out/rpshi/c3.txt &&
BENCH_ARGS="--config c5" timeout -k 10 300 sh tools/ab_env.sh PPO_OUTHEAD_RPS 16 32 > gpurun_out/rpshi/c5.txt 2>&1 && cat gpurun_out/rpshi/c5.txt &&
PPO_COMM_SELF=1 BENCH_ARGS="--emulate-world 8" timeout -k 10 300 sh tools/ab_env.sh PPO_OUTHEAD_RPS 16 32 > gpurun_out/rpshi/shard.txt 2>&1 && cat gpurun_out/rpshi/shard.txt
