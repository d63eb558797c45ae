#!/bin/sh
# r04_c5_ab.sh TAG — same-box A/Bs at C5 (bf16): grad_W TN tile width and split-K workgroup target
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
BENCH_ARGS="--config c5" sh tools/ab_env.sh PPO_G16_TN_BN 256 128 > $O/ab_bn.txt 2>&1 || { cat $O/ab_bn.txt; exit 1; }
cat $O/ab_bn.txt
BENCH_ARGS="--config c5" sh tools/ab_env.sh PPO_G16_TN_TARGET 256 128 512 > $O/ab_target.txt 2>&1 || { cat $O/ab_target.txt; exit 1; }
cat $O/ab_target.txt
