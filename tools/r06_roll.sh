#!/bin/sh
# r06_roll.sh TAG — C4 at B = 64: weight-gradient tiles with a rolling prefetch (variant roll, CLU_GW_ROLL=1) vs
# one tile's loads at a time (libppo): stamps of each, then update times interleaved twice
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
V=$R/ppo.c_amd/lib/variants
for v in def roll; do
  L=$R/ppo.c_amd/lib/libppo.so; [ $v = def ] || L=$V/libppo_$v.so
  PPO_LIB=$L PPO_CLUSTER_STAMPS=1 timeout -k 10 200 python bench.py --config c4 --batch 64 --steps 1 --warmup 1 \
      --no-cpu-baseline --no-rollout --no-kernel-events > $O/st_$v.log 2>&1 || exit 1
done
for i in 1 2; do for v in roll def; do
  L=$R/ppo.c_amd/lib/libppo.so; [ $v = def ] || L=$V/libppo_$v.so
  PPO_LIB=$L timeout -k 10 200 python bench.py --config c4 --batch 64 --steps 2 --warmup 1 \
      --no-cpu-baseline --no-rollout --no-kernel-events > $O/t_${v}_$i.log 2>&1 || exit 1
done; done
