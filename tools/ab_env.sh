#!/bin/sh
# ab_env.sh TAG VAR — one-box A/B of an environment switch: bench.py lines (C4, G = 8 shard, C3) with
# VAR=0 (A) and VAR=1 (B), run A B A B so box drift shows.  Output under gpurun_out/TAG/.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
for rep in 1 2; do
    for L in A B; do
        if [ $L = A ]; then V=0; else V=1; fi
        env $2=$V timeout -k 10 200 python bench.py --no-cpu-baseline --no-rollout 2>/dev/null | tail -1 > $O/c4_${L}$rep.json || exit 1
        env $2=$V PPO_COMM_SELF=1 timeout -k 10 200 python bench.py --emulate-world 8 --no-cpu-baseline --no-rollout 2>/dev/null | tail -1 > $O/shard8_${L}$rep.json || exit 1
        env $2=$V timeout -k 10 200 python bench.py --config c3 --no-cpu-baseline --no-rollout 2>/dev/null | tail -1 > $O/c3_${L}$rep.json || exit 1
    done
done
python - "$O" <<'PY'
import json, sys, glob, os
o = sys.argv[1]
for f in sorted(glob.glob(os.path.join(o, "*.json"))):
    try:
        print(f"{os.path.basename(f):16s} {json.load(open(f))['ms_per_step']:8.2f} ms")
    except Exception as e:
        print(f, "unreadable", e)
PY
