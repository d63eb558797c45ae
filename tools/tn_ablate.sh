#!/bin/sh
# tn_ablate.sh TAG — bf16 DMA TN grad_W (C5 shape) per libppo variant: ablations (1 no MFMA, 2 no
# epilogue stores, 4 no DMA after the prologue, 7 all three) and the direct-store epilogue, into
# gpurun_out/TAG/tn_ablate.txt (each line includes the slab reduce launch)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
for L in lib/libppo.so lib/variants/libppo_tndirect.so lib/variants/libppo_tnab1.so lib/variants/libppo_tnab2.so \
         lib/variants/libppo_tnab4.so lib/variants/libppo_tnab7.so; do
  echo "$L" >> $O/tn_ablate.txt
  PPO_LIB=$R/ppo.c_amd/$L timeout -k 10 100 python3 $R/tools/tn16_bench.py 16384 1024 1024 >> $O/tn_ablate.txt 2>&1 || exit 1
done
