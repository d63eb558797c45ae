#!/bin/sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
for rep in 1 2; do
  for v in 0 1; do
    if [ $v = 1 ]; then export PPO_COMM_SELF=1; else unset PPO_COMM_SELF; fi
    echo "COMM_SELF=$v $(timeout -k 10 200 python bench.py --emulate-world 8 --no-cpu-baseline --no-rollout 2>/dev/null | tail -1 | python -c 'import json,sys; print(round(json.load(sys.stdin)["ms_per_step"],2))')"
    echo "COMM_SELF=$v serial $(PPO_SERIAL=1 timeout -k 10 200 python bench.py --emulate-world 8 --no-cpu-baseline --no-rollout 2>/dev/null | tail -1 | python -c 'import json,sys; print(round(json.load(sys.stdin)["ms_per_step"],2))')"
  done
done
