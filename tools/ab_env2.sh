#!/bin/sh
# ab_env2.sh TAG "BENCH ARGS" "ENV=VAL" — bench ms per update with and without one environment setting,
# interleaved twice on one box, into gpurun_out/TAG/ab.txt
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; ARGS=$2; EV=$3
mkdir -p $O
for rep in 1 2; do
  timeout -k 10 200 python3 $R/bench.py --no-cpu-baseline --no-rollout --no-kernel-events $ARGS | grep '^{' | python3 -c "import json,sys; print('default', '$ARGS', round(json.loads(sys.stdin.read())['ms_per_step'],2))" >> $O/ab.txt || exit 1
  env $EV timeout -k 10 200 python3 $R/bench.py --no-cpu-baseline --no-rollout --no-kernel-events $ARGS | grep '^{' | python3 -c "import json,sys; print('$EV', '$ARGS', round(json.loads(sys.stdin.read())['ms_per_step'],2))" >> $O/ab.txt || exit 1
done
