#!/bin/sh
# r06_serial64.sh TAG — C4 at B = 64 with the value and policy phases one after the other (PPO_SERIAL=1):
# per-workgroup release stamps of each phase alone, then the update time, beside the concurrent default
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
PPO_SERIAL=1 PPO_CLUSTER_STAMPS=2 timeout -k 10 200 python bench.py --config c4 --batch 64 --steps 1 --warmup 1 \
    --no-cpu-baseline --no-rollout --no-kernel-events > $O/st_serial.log 2>&1 || exit 1
PPO_SERIAL=1 timeout -k 10 200 python bench.py --config c4 --batch 64 --steps 2 --warmup 1 \
    --no-cpu-baseline --no-rollout --no-kernel-events > $O/t_serial.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --config c4 --batch 64 --steps 2 --warmup 1 \
    --no-cpu-baseline --no-rollout --no-kernel-events > $O/t_def.log 2>&1 || exit 1
