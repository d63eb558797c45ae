#!/bin/sh
# fused value head rows per wave slot (PPO_OUTHEAD_RPS) at C4 (32,768-row minibatches)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 500 sh tools/ab_env.sh PPO_OUTHEAD_RPS 16 8 32 4 > gpurun_out/rps_c4.txt 2>&1; rc=$?; cat gpurun_out/rps_c4.txt; exit $rc
