#!/bin/sh
# r04_stride_stamps.sh TAG — C4 B = 64 value-step stamps at PPO_CLUSTER_STRIDE 1 / 2 / 4, three rounds
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
for rep in 1 2 3; do
for st in 1 2 4; do
  PPO_CLUSTER_STRIDE=$st PPO_CLUSTER_STAMPS=1 timeout -k 10 200 python bench.py --config c4 --batch 64 --steps 1 --warmup 0 --no-cpu-baseline --no-rollout --no-kernel-events > $O/st.log 2>&1 || { tail -5 $O/st.log; exit 1; }
  echo "stride $st: $(grep 'cluster_deep value' $O/st.log | head -1 | sed 's/.*| //') $(grep 'cluster_deep value' $O/st.log | head -1 | grep -o 'bar A [0-9.]*') $(grep 'cluster_deep policy' $O/st.log | head -1 | sed 's/.*| /policy /')"
done
done
