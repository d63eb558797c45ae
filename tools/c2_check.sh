#!/bin/sh
# C2 tiny-path check: parity tests, C2 bench (specialised vs generic kernel), phase stamps
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_tiny.py tests/test_gpu_production.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 200 python3 bench.py --config c2 --no-cpu-baseline --no-rollout > $O/c2.json 2>&1 || exit 1
PPO_TINY_STAMPS=1 timeout -k 10 200 python3 bench.py --config c2 --no-cpu-baseline --no-rollout --no-kernel-events --steps 1 --warmup 1 > $O/c2_stamps.txt 2>&1
