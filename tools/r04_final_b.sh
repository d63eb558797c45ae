#!/bin/sh
# r04_final_b.sh TAG — round-end check part 2: every config's bench line on one box (C3, C2, C5 shard,
# the G = 8 C4 shard, C3 and C4 at B = 64)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
run() { n=$1; shift; timeout -k 10 300 "$@" > $O/$n.json 2> $O/$n.err || { tail -5 $O/$n.err; exit 1; }
        python3 -c "import json; d=json.load(open('$O/$n.json')); print('$n', round(d['ms_per_step'],2), 'ms', round(d['value']), d['unit'], 'frac', round(d['roofline']['frac'],3))"; }
run c3 python3 bench.py --config c3 --no-rollout
run c2 python3 bench.py --config c2 --no-rollout
run c5 python3 bench.py --config c5 --no-cpu-baseline --no-rollout
run shard8 env PPO_COMM_SELF=1 python3 bench.py --emulate-world 8 --no-cpu-baseline --no-rollout
run c3b64 python3 bench.py --config c3 --batch 64 --no-rollout --steps 3 --warmup 1
run c4b64 python3 bench.py --config c4 --batch 64 --no-rollout --steps 2 --warmup 1
