#!/bin/bash
# ab_tiny.sh TAG — C2 single-workgroup path: parity tests, per-phase stamps and a same-box A/B of
# libppo builds (lib/libppo_tinybase.so = the previous tiny kernel)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_tiny.py -x -q --timeout 200 --timeout-method thread > $O/test.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/test.log
case $rc in 124|134|137|139) exit 1;; esac
PPO_TINY_STAMPS=1 timeout -k 10 120 python bench.py --config c2 --steps 1 --warmup 0 --no-cpu-baseline --no-rollout > $O/stamps.log 2>&1 || exit 1
BENCH_ARGS="--config c2 --steps 10" sh tools/ab_lib.sh ppo.c_amd/lib/libppo_tinybase.so ppo.c_amd/lib/libppo.so > $O/ab.log 2>&1 || exit 1
