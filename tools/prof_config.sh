#!/bin/sh
# prof_config.sh OUT CONFIG [bench args...] — bench line + rocprofv3 kernel trace/stats of one serial
# update of CONFIG, into gpurun_out/OUT/ (the trace's last update: tools/trace_update.py)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; C=$2; shift 2
mkdir -p $O
timeout -k 10 200 python3 $R/bench.py --config $C --no-cpu-baseline "$@" > $O/$C.log 2>&1
cd /tmp && export TMPDIR=/tmp
PPO_SERIAL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$C -o run --output-format csv -- python3 $R/bench.py --config $C --steps 1 --warmup 1 --no-cpu-baseline --no-kernel-events --no-rollout "$@" > $O/prof_$C.log 2>&1
