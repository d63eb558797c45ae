#!/bin/sh
# r04_stamps_ab.sh TAG LIB... — per-sub-phase stamps of the C4 B = 64 phases for each libppo build, same box
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; shift
mkdir -p $O
cd $R
for rep in 1 2; do
for L in "$@"; do
  PPO_LIB=$L PPO_CLUSTER_STAMPS=1 timeout -k 10 200 python bench.py --config c4 --batch 64 --steps 1 --warmup 0 --no-cpu-baseline --no-rollout --no-kernel-events > $O/st.log 2>&1 || { tail -5 $O/st.log; exit 1; }
  echo "== $L"; grep cluster_deep $O/st.log | head -2
done
done
