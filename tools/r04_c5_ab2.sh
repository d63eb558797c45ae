#!/bin/sh
# r04_c5_ab2.sh TAG — C5: the 256×128 grad_W TN tile at split targets 256 / 128 vs the 256×256 default
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
for rep in 1 2; do
  for v in "PPO_G16_TN_BN=256" "PPO_G16_TN_BN=128" "PPO_G16_TN_BN=128 PPO_G16_TN_TARGET=128" "PPO_G16_TN_BN=128 PPO_G16_TN_TARGET=384"; do
    env $v timeout -k 10 120 python3 bench.py --config c5 --no-cpu-baseline --no-rollout --no-kernel-events | grep '^{' | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', round(d['ms_per_step'],2))" || exit 1
  done
done
