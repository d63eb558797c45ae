#!/bin/sh
# fused heads rows per wave slot (PPO_OUTHEAD_RPS) at C3 (8,192-row minibatches: 128 workgroups at 16)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
BENCH_ARGS="--config c3" timeout -k 10 500 sh tools/ab_env.sh PPO_OUTHEAD_RPS 16 8 4 2 1 > gpurun_out/rps_c3.txt 2>&1; rc=$?; cat gpurun_out/rps_c3.txt; exit $rc
