#!/bin/sh
# r06_shift.sh TAG — C4 at B = 64, concurrent phases: the policy phase's barrier counters / hand-off buffers
# moved against the value phase's (PPO_CLUSTER_SHIFT_CTR / _WS): release stamps, then update times
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
run() {  # name, env...
  n=$1; shift
  env "$@" PPO_CLUSTER_STAMPS=2 timeout -k 10 200 python bench.py --config c4 --batch 64 --steps 1 --warmup 1 \
      --no-cpu-baseline --no-rollout --no-kernel-events > $O/st_$n.log 2>&1 || exit 1
  env "$@" timeout -k 10 200 python bench.py --config c4 --batch 64 --steps 2 --warmup 1 \
      --no-cpu-baseline --no-rollout --no-kernel-events > $O/t_$n.log 2>&1 || exit 1
}
run base PPO_NONE=1
run ctr2k PPO_CLUSTER_SHIFT_CTR=2048
run ws32k PPO_CLUSTER_SHIFT_WS=32768
run both PPO_CLUSTER_SHIFT_CTR=2048 PPO_CLUSTER_SHIFT_WS=32768
