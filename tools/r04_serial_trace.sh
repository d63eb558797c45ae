#!/bin/sh
# r04_serial_trace.sh TAG [bench args...] — rocprofv3 --kernel-trace --stats of ONE serialised
# (PPO_SERIAL=1) C4 update of HEAD, plus the default bench line on the same box
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; shift
mkdir -p $O
cd $R
timeout -k 10 240 python bench.py "$@" > $O/bench.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
PPO_SERIAL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-kernel-events --no-rollout "$@" > $O/prof.log 2>&1 || exit 1
python3 $R/tools/trace_update.py $(ls $O/prof/*/run_kernel_trace.csv $O/prof/run_kernel_trace.csv 2>/dev/null | head -1) --top 40 > $O/breakdown.txt 2>&1
