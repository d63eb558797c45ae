#!/bin/sh
# r05_phase_gather_check.sh — GPU tests touching the minibatch gather + bench lines (shard, C3, C4)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/r05pg
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_index.py tests/test_gpu_ops.py tests/test_gpu_update.py tests/test_gpu_value_fold.py tests/test_gpu_production.py tests/test_gpu_dp_shards.py > $O/tests.log 2>&1
for rep in 1 2; do
  PPO_COMM_SELF=1 timeout -k 10 200 python bench.py --emulate-world 8 --no-cpu-baseline --no-rollout 2>/dev/null | tail -1 > $O/shard8_$rep.json
  timeout -k 10 200 python bench.py --config c3 --no-cpu-baseline --no-rollout 2>/dev/null | tail -1 > $O/c3_$rep.json
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-rollout 2>/dev/null | tail -1 > $O/c4_$rep.json
done
for f in $O/*.json; do python -c "import json,sys; d=json.load(open('$f')); print('$f'.split('/')[-1], d['ms_per_step'])"; done
