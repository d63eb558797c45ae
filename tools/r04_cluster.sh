#!/bin/sh
# r04_cluster.sh TAG [ENV-VARIANTS...] — B = 64 cluster phase: parity tests, per-sub-phase stamps,
# C3 B = 64 bench (default settings, then once per extra "VAR=value" variant)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
shift
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_cluster.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
PPO_CLUSTER_STAMPS=1 timeout -k 10 120 python bench.py --config c3 --batch 64 --steps 1 --warmup 1 > $O/stamps.log 2>&1 || exit 1
grep cluster $O/stamps.log | head -2
for V in default "$@"; do
  timeout -k 10 200 env $([ $V = default ] || echo $V) python bench.py --config c3 --batch 64 --steps 3 --warmup 1 > $O/c3b64_$V.json 2>$O/c3b64_$V.err || exit 1
  python3 -c "import json,sys; d=json.load(open('$O/c3b64_$V.json')); print('c3 b64 $V ms/update', d['ms_per_step'])"
done
