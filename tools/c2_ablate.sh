#!/bin/sh
# C2 tiny-kernel phase stamps per ablation variant (tools/build_variant.sh c2abN -DPPO_C2_AB=N tiny)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
for L in lib/libppo.so lib/variants/libppo_c2ab1.so lib/variants/libppo_c2ab2.so lib/variants/libppo_c2ab4.so lib/variants/libppo_c2ab8.so; do
  echo "$L" >> $O/c2_ablate.txt
  PPO_LIB=$R/ppo.c_amd/$L PPO_TINY_STAMPS=1 timeout -k 10 100 python3 $R/bench.py --config c2 --no-cpu-baseline --no-rollout --no-kernel-events --steps 1 --warmup 1 2>&1 | grep "tiny.*value\|sub-phases" | head -2 >> $O/c2_ablate.txt || exit 1
done
