#!/bin/sh
# r04_batch2.sh TAG — cluster tests, then C4 and C3 B = 64 (stamps + bench)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_cluster.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log; grep "steps vs oracle" $O/tests.log
sh tools/r04_deep.sh $1 || exit 1
PPO_CLUSTER_STAMPS=1 timeout -k 10 120 python bench.py --config c3 --batch 64 --steps 1 --warmup 1 --no-cpu-baseline > $O/c3stamps.log 2>&1 || exit 1
grep "cluster " $O/c3stamps.log | head -2
timeout -k 10 200 python bench.py --config c3 --batch 64 --steps 3 --warmup 1 > $O/c3b64.json 2>$O/c3b64.err || exit 1
python3 -c "import json; d=json.load(open('$O/c3b64.json')); print('c3 b64 ms/update', d['ms_per_step'])"
