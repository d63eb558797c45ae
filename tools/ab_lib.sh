#!/bin/sh
# ab_lib.sh LIB1 LIB2 ... — bench ms per update with each libppo build (PPO_LIB), interleaved twice
# on one box; BENCH_ARGS passes bench options (e.g. "--config c5")
R=${GRAFT_REPO_ROOT:-$(pwd)}
for rep in 1 2; do
  for L in "$@"; do
    PPO_LIB=$L timeout -k 10 120 python3 $R/bench.py --no-cpu-baseline --no-rollout --no-kernel-events $BENCH_ARGS | grep '^{' | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$L', round(d['ms_per_step'],2))" || exit 1
  done
done
