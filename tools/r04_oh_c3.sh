#!/bin/sh
# C3 fused heads: exp(log σ) hoisted (working tree) vs HEAD's out_head.hip, same box; rows-per-slot
# scan at C3; then the fused-head / update / production GPU tests
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/ohc3
BENCH_ARGS="--config c3" timeout -k 10 400 sh tools/ab_lib.sh $R/ppo.c_amd/lib/libppo.so $R/ppo.c_amd/lib/variants/libppo_oh_old.so > gpurun_out/ohc3/lib.txt 2>&1 && cat gpurun_out/ohc3/lib.txt &&
BENCH_ARGS="--config c3" timeout -k 10 500 sh tools/ab_env.sh PPO_OUTHEAD_RPS 16 8 4 2 > gpurun_out/ohc3/rps.txt 2>&1 && cat gpurun_out/ohc3/rps.txt &&
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_update.py tests/test_gpu_production.py -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/ohc3/tests.txt 2>&1; rc=$?; tail -3 gpurun_out/ohc3/tests.txt; exit $rc
