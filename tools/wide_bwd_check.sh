#!/bin/sh
# wide (A = 17) output-layer backward: parity tests, C4 with / without it
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_update.py tests/test_gpu_production.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
for rep in 1 2; do
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-rollout --no-kernel-events | grep '^{' | python3 -c "import json,sys; print('wide-bwd', round(json.loads(sys.stdin.read())['ms_per_step'],2))" >> $O/ab.txt || exit 1
  PPO_NO_WIDE_BWD=1 timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-rollout --no-kernel-events | grep '^{' | python3 -c "import json,sys; print('pair', round(json.loads(sys.stdin.read())['ms_per_step'],2))" >> $O/ab.txt || exit 1
done
timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-rollout > $O/c4.json 2>&1
