#!/bin/sh
# ab_env.sh VAR V1 V2 ... — C4 bench ms per update with environment variable VAR set to each value,
# interleaved twice (same box)
R=${GRAFT_REPO_ROOT:-$(pwd)}
VAR=$1; shift
for rep in 1 2; do
  for v in "$@"; do
    env $VAR=$v timeout -k 10 120 python3 $R/bench.py --no-cpu-baseline --no-rollout --no-kernel-events $BENCH_ARGS | grep '^{' | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$VAR=$v', round(d['ms_per_step'],2))" || exit 1
  done
done
