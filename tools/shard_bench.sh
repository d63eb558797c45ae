#!/bin/sh
# shard_bench.sh TAG [G...] — rank 0's shard of a G-way split of the C4 rollout on one GPU
# (bench.py --emulate-world G: E/G envs, B/G rows per step) through a one-rank RCCL communicator
# (PPO_COMM_SELF=1: every gradient all-reduce on the comm stream as at world > 1), then a rocprofv3
# kernel trace of one G=8 shard update (comm-stream share).  Lines into gpurun_out/TAG/.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; shift
mkdir -p $O
for G in ${@:-2 4 8}; do
  PPO_COMM_SELF=1 timeout -k 10 200 python3 $R/bench.py --emulate-world $G --no-cpu-baseline > $O/shard$G.json 2> $O/shard$G.err
done
cd /tmp && export TMPDIR=/tmp
PPO_COMM_SELF=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof8 -o run --output-format csv -- python3 $R/bench.py --emulate-world 8 --steps 2 --warmup 1 --no-cpu-baseline --no-kernel-events --no-rollout > $O/prof8.log 2>&1
