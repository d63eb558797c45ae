#!/bin/sh
# r04_deep.sh TAG [ENV-VARIANTS...] — C4 networks at B = 64 on the 32-workgroup phase: per-sub-phase
# stamps, then the C4 B = 64 bench (default settings, then once per extra "VAR=value" variant)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
shift
mkdir -p $O
cd $R
PPO_CLUSTER_STAMPS=1 timeout -k 10 200 python bench.py --config c4 --batch 64 --steps 1 --warmup 0 --no-cpu-baseline > $O/stamps.log 2>&1 || { tail -5 $O/stamps.log; exit 1; }
grep cluster_deep $O/stamps.log | head -2
for V in default "$@"; do
  timeout -k 10 300 env $([ $V = default ] || echo $V) python bench.py --config c4 --batch 64 --steps 2 --warmup 1 > $O/c4b64_$V.json 2>$O/c4b64_$V.err || exit 1
  python3 -c "import json,sys; d=json.load(open('$O/c4b64_$V.json')); print('c4 b64 $V ms/update', d['ms_per_step'])"
done
