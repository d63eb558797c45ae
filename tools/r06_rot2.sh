#!/bin/sh
# r06_rot2.sh TAG — C4 at B = 64: per-workgroup exit lateness with the slices as launched and rotated by 8,
# then the update time (no stamps) at slice rotations 0, 8, 16, 24, 4, 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
for r in 0 8; do
  PPO_CLUSTER_ROT=$r PPO_CLUSTER_STAMPS=2 timeout -k 10 200 python bench.py --config c4 --batch 64 --steps 1 --warmup 1 \
      --no-cpu-baseline --no-rollout --no-kernel-events > $O/c4b64_rot$r.log 2>&1 || exit 1
done
for r in 0 8 16 24 4 2; do
  PPO_CLUSTER_ROT=$r timeout -k 10 200 python bench.py --config c4 --batch 64 --steps 2 --warmup 1 \
      --no-cpu-baseline --no-rollout --no-kernel-events > $O/c4b64_t_rot$r.log 2>&1 || exit 1
done
