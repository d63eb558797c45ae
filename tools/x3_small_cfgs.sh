#!/bin/sh
# x3_small_cfgs.sh — small-tile shape candidates (diagnostic build, cfgs 6-9: 64x64 over 2 waves, 128x64
# over 4 waves) against cfg 4 (64x64 over 4 waves) at the G = 8 shard and C3 shapes, then the barrier-skip
# ablation (ABL 128) of cfg 4; run twice so box drift shows
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
D=$R/ppo.c_amd/lib/variants/libppo_diag.so
for rep in 1 2; do
  for s in "0 4096 512 512" "1 4096 512 512" "0 4096 376 512" "0 8192 256 256" "1 8192 256 256"; do
    for c in 4 6 7 8 9; do
      PPO_LIB=$D GEMM_ENGINE=x3 timeout -k 5 60 python tools/gemm_one.py $s $c 100
    done
    echo "ablate 128: $(PPO_LIB=$D PPO_X3_ABLATE=128 GEMM_ENGINE=x3 timeout -k 5 60 python tools/gemm_one.py $s 4 100)"
  done
  # grad_W (split-K + slab reduce): 128x128 two k-groups (cfg 3, production) vs 64x64 (cfg 4)
  for s in "2 4096 512 512" "2 8192 256 256" "2 4096 376 512"; do
    for c in 3 4; do
      PPO_LIB=$D GEMM_ENGINE=x3 timeout -k 5 60 python tools/gemm_one.py $s $c 100
    done
  done
done
