#!/bin/sh
# r06_fnwg.sh TAG — policy_out_fused_kernel's grid at C4 (PPO_POLICY_FUSED=1): 256 / 512 / 1024 workgroups
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
for g in 256 512 1024 2048; do
  PPO_POLICY_FUSED=1 PPO_FUSED_NWG=$g timeout -k 10 240 python bench.py --no-cpu-baseline --no-rollout --steps 2 --warmup 1 > $O/c4_g$g.log 2>&1 || exit 1
done
