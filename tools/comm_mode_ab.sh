#!/bin/sh
# comm_mode_ab.sh — the G = 8 shard line (PPO_COMM_SELF=1, one-rank RCCL) under the diagnostic comm modes of
# lib/variants/libppo_commdiag.so: 0 = comm stream + events (shipped), 1 = all-reduce on the issuing stream,
# 2 = events only (no collective); and without a communicator
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export PPO_LIB=$R/ppo.c_amd/lib/variants/libppo_commdiag.so
for rep in 1 2; do
  for m in 0 1 2; do
    for ser in 0 1; do
      if [ $ser = 1 ]; then export PPO_SERIAL=1; else unset PPO_SERIAL; fi
      echo "mode $m serial $ser $(PPO_COMM_MODE=$m PPO_COMM_SELF=1 timeout -k 10 200 python bench.py --emulate-world 8 --no-cpu-baseline --no-rollout 2>/dev/null | tail -1 | python -c 'import json,sys; print(round(json.load(sys.stdin)["ms_per_step"],2))')"
    done
  done
  unset PPO_SERIAL
  echo "no comm $(timeout -k 10 200 python bench.py --emulate-world 8 --no-cpu-baseline --no-rollout 2>/dev/null | tail -1 | python -c 'import json,sys; print(round(json.load(sys.stdin)["ms_per_step"],2))')"
done
