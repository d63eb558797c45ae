#!/bin/sh
# r06_rot.sh TAG — C4 at B = 64 with per-workgroup barrier stamps, the hidden slices owned by the workgroups
# as launched (rot 0) and rotated by one and by eight (PPO_CLUSTER_ROT): a slow workgroup that follows its
# slice is data-placed, one that stays is hardware-placed
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
for r in 0 1 8; do
  PPO_CLUSTER_ROT=$r PPO_CLUSTER_STAMPS=2 timeout -k 10 200 python bench.py --config c4 --batch 64 --steps 2 --warmup 1 \
      --no-cpu-baseline --no-rollout --no-kernel-events > $O/c4b64_rot$r.log 2>&1 || exit 1
done
