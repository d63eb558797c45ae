#!/bin/sh
# r06_ab.sh TAG — the -m gpu suite, then C4 A/B alternating (default vs PPO_X0_COPY=1), then the B = 64 PMC pass
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 240 python bench.py --no-cpu-baseline --no-rollout > $O/c4_$i.log 2>&1 || exit 1
  PPO_X0_COPY=1 timeout -k 10 240 python bench.py --no-cpu-baseline --no-rollout > $O/c4_x0copy_$i.log 2>&1 || exit 1
done
sh tools/pmc_c4b64.sh $1
