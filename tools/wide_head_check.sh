#!/bin/sh
# fused A = 17 policy head + wide backward: parity tests, C4 default vs PPO_NO_WIDE_HEAD=1 (separate head,
# wide backward) vs PPO_NO_WIDE_BWD=1 (separate head, paired GEMM), and C3
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_update.py tests/test_gpu_production.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
for rep in 1 2; do
  for ev in "X=0" "PPO_NO_WIDE_HEAD=1" "PPO_NO_WIDE_BWD=1"; do
    env $ev timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-rollout --no-kernel-events | grep '^{' | python3 -c "import json,sys; print('$ev', round(json.loads(sys.stdin.read())['ms_per_step'],2))" >> $O/ab.txt || exit 1
  done
done
timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-rollout > $O/c4.json 2>&1 || exit 1
timeout -k 10 200 python3 bench.py --config c3 --no-cpu-baseline --no-rollout > $O/c3.json 2>&1
