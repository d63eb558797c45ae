#!/bin/sh
# gpu_check.sh — one GPU-box pass: the -m gpu suite, then C4 / C2 (+ single-workgroup phase stamps) / C3 / C5 bench lines into gpurun_out/r1/
set -e
O=gpurun_out/r1
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
timeout -k 10 120 python bench.py --no-cpu-baseline > $O/c4.log 2>&1
timeout -k 10 120 python bench.py --config c2 --no-cpu-baseline > $O/c2.log 2>&1
PPO_TINY_STAMPS=1 timeout -k 10 120 python bench.py --config c2 --steps 1 --warmup 1 --no-cpu-baseline --no-rollout > $O/c2_stamps.log 2>&1
timeout -k 10 120 python bench.py --config c3 --no-cpu-baseline > $O/c3.log 2>&1
timeout -k 10 200 python bench.py --config c5 --no-cpu-baseline > $O/c5.log 2>&1
