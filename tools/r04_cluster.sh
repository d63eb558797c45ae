#!/bin/sh
# r04_cluster.sh TAG — B = 64 cluster phase: parity tests, per-sub-phase stamps, C3 B = 64 bench
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_cluster.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
PPO_CLUSTER_STAMPS=1 timeout -k 10 120 python bench.py --config c3 --batch 64 --steps 1 --warmup 1 > $O/stamps.log 2>&1 || exit 1
grep cluster $O/stamps.log | head -2
timeout -k 10 200 python bench.py --config c3 --batch 64 --steps 3 --warmup 1 > $O/c3b64.json 2>$O/c3b64.err || exit 1
python3 -c "import json,sys; d=json.load(open('$O/c3b64.json')); print('c3 b64 ms/update', d['ms_per_step'])"
