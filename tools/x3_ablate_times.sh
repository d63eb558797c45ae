#!/bin/sh
# x3_ablate_times.sh — µs per launch of the C4 x3 products (forward, grad_x, grad_W at 512x512,
# automatic configuration) with parts of the kernel removed (PPO_X3_ABLATE; diagnostic build
# `tools/build_variant.sh diag -DPPO_X3_DIAG gemm_x3`): 0 none, 1 MFMAs, 2 split + LDS stores,
# 4 epilogue stores, 8 global loads, 64 the split alone
R=$GRAFT_REPO_ROOT
export PPO_LIB=${PPO_LIB:-$R/ppo.c_amd/lib/variants/libppo_diag.so}
for op in 0 1 2; do
  for ab in 0 1 2 4 8 64; do
    PPO_X3_ABLATE=$ab GEMM_ENGINE=x3 timeout -k 10 60 python3 $R/tools/gemm_one.py $op 32768 512 512 -1 50 | sed "s/^/ablate=$ab /" || exit 1
  done
done
