#!/bin/sh
# r06_fabl.sh TAG — timing ablations of policy_out_fused_kernel (results wrong): 1 no μ MFMA, 2 no head,
# 4 no gx / gW3 rows, 8 no h loads, 15 none of them; C4 by_shape
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
timeout -k 10 240 python bench.py --no-cpu-baseline --no-rollout --steps 2 --warmup 1 > $O/abl0.log 2>&1 || exit 1
for v in 1 2 4 8 15; do
  PPO_LIB=$R/ppo.c_amd/lib/variants/libppo_fabl$v.so timeout -k 10 240 python bench.py --no-cpu-baseline --no-rollout --steps 2 --warmup 1 > $O/abl$v.log 2>&1 || exit 1
done
