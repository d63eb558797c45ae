#!/bin/sh
# ab_bench.sh TAG "BENCH ARGS" LIB... — bench ms per update per libppo build (PPO_LIB), interleaved
# twice on one box, into gpurun_out/TAG/ab.txt
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; ARGS=$2; shift 2
mkdir -p $O
for rep in 1 2; do
  for L in "$@"; do
    PPO_LIB=$L timeout -k 10 200 python3 $R/bench.py --no-cpu-baseline --no-rollout --no-kernel-events $ARGS | grep '^{' | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$L', '$ARGS', round(d['ms_per_step'],2))" >> $O/ab.txt || exit 1
  done
done
