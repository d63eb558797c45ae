#!/bin/sh
# final_configs.sh TAG — every config's bench line on one box (C3, C2, the C5 shard, the G = 8 C4 shard,
# C3 and C4 at B = 64) into gpurun_out/TAG/ (BASELINE.md §3 via tools/results_table.py)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
run() { n=$1; shift; timeout -k 10 300 "$@" > $O/$n.json 2> $O/$n.err || { tail -5 $O/$n.err; exit 1; }
        python3 -c "import json; d=[l for l in open('$O/$n.json') if l.startswith('{')][-1]; d=json.loads(d); print('$n', round(d['ms_per_step'],2), 'ms', round(d['value']), d['unit'], 'frac', round(d['roofline']['frac'],3))"; }
run c3 python3 bench.py --config c3 --no-rollout
run c2 python3 bench.py --config c2 --no-rollout
run c5 python3 bench.py --config c5 --no-cpu-baseline --no-rollout
run shard8 env PPO_COMM_SELF=1 python3 bench.py --emulate-world 8 --no-cpu-baseline --no-rollout
run c3b64 python3 bench.py --config c3 --batch 64 --no-rollout --steps 3 --warmup 1
run c4b64 python3 bench.py --config c4 --batch 64 --no-rollout --steps 2 --warmup 1
