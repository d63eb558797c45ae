#!/bin/sh
# comm_ab.sh — the G = 8 shard line (PPO_COMM_SELF=1: a one-rank RCCL communicator) with the gradient
# all-reduces in stream order (default) and on the comm stream behind event pairs (PPO_COMM_ASYNC=1),
# and without a communicator; concurrent and serial loops, A B A B
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
b() { timeout -k 10 200 python bench.py --emulate-world 8 --no-cpu-baseline --no-rollout 2>/dev/null | tail -1 | python -c 'import json,sys; print(round(json.load(sys.stdin)["ms_per_step"],2))'; }
for rep in 1 2; do
  echo "async   $(PPO_COMM_ASYNC=1 PPO_COMM_SELF=1 b)   serial $(PPO_SERIAL=1 PPO_COMM_ASYNC=1 PPO_COMM_SELF=1 b)"
  echo "inline  $(PPO_COMM_SELF=1 b)   serial $(PPO_SERIAL=1 PPO_COMM_SELF=1 b)"
  echo "no comm $(b)   serial $(PPO_SERIAL=1 b)"
done
