#!/bin/sh
# g16_ablate.sh [VARIANTS] — the double-buffered bf16 GEMM (cfg 9) at the C5 shape under the
# PPO_G16_ABLATE diagnostic builds (tools/build_variant.sh g16abN -DPPO_G16_ABLATE=N gemm16) next to
# production (0)
R=${GRAFT_REPO_ROOT:-$(pwd)}
for v in ${1:-0 1 2 4 8 16 6 12}; do
  if [ $v = 0 ]; then L=$R/ppo.c_amd/lib/libppo.so; else L=$R/ppo.c_amd/lib/variants/libppo_g16ab$v.so; fi
  echo "ablate=$v"
  PPO_LIB=$L NO_GRADW=1 timeout -k 10 60 python3 $R/tools/gemm16_sweep.py --cfgs 9 || exit 1
done
