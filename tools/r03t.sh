#!/bin/sh
# round-3 check: tiny C2 kernel + bf16 DMA TN (tests, C2 / C5 benches, phase stamps)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_tiny.py tests/test_gpu_production.py tests/test_gpu_bf16.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 200 python3 bench.py --config c2 --no-cpu-baseline --no-rollout > $O/c2.json 2>&1 || exit 1
PPO_TINY_GENERIC=1 timeout -k 10 200 python3 bench.py --config c2 --no-cpu-baseline --no-rollout --no-kernel-events > $O/c2_generic.json 2>&1 || exit 1
PPO_TINY_STAMPS=1 timeout -k 10 200 python3 bench.py --config c2 --no-cpu-baseline --no-rollout --no-kernel-events --steps 1 --warmup 1 > $O/c2_stamps.txt 2>&1 || exit 1
timeout -k 10 120 python3 tools/tn16_bench.py > $O/tn.txt 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --config c5 --no-cpu-baseline --no-rollout > $O/c5.json 2>&1 || exit 1
PPO_G16_TN=0 timeout -k 10 300 python3 bench.py --config c5 --no-cpu-baseline --no-rollout --no-kernel-events > $O/c5_off.json 2>&1
