#!/bin/sh
# c4b64_placement.sh TAG — C4 at the reference's B = 64 (cluster_deep.hip phases): per-update time,
# per-sub-phase stamps and each workgroup's XCC / SE / CU, for several runs and placement strides
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
export PPO_CLUSTER_STAMPS=1
for st in ${STRIDES:-2 2 2 1 1 4 4 8}; do
    PPO_CLUSTER_STRIDE=$st timeout -k 10 120 python bench.py --batch 64 --steps 1 --warmup 1 --no-cpu-baseline \
        --no-rollout --no-kernel-events > $O/out.json 2> $O/err.txt || exit 1
    ms=$(python3 -c "import json;print(json.loads([l for l in open('$O/out.json') if l.startswith('{')][-1])['ms_per_step'])")
    echo "stride $st: $ms ms per update"
    grep "cluster_deep" $O/err.txt | tail -4
done
