#!/bin/sh
# r04_shard_trace.sh TAG — a kernel trace of one G = 8 shard update (concurrent, as timed) and a serial one
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
PPO_COMM_SELF=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/conc -o run --output-format csv -- python3 $R/bench.py --emulate-world 8 --steps 1 --warmup 1 --no-cpu-baseline --no-kernel-events --no-rollout > $O/conc.log 2>&1 || exit 1
python3 $R/tools/trace_update.py $(ls $O/conc/*/run_kernel_trace.csv $O/conc/run_kernel_trace.csv 2>/dev/null | head -1) --top 30 > $O/conc_breakdown.txt 2>&1
PPO_SERIAL=1 PPO_COMM_SELF=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/ser -o run --output-format csv -- python3 $R/bench.py --emulate-world 8 --steps 1 --warmup 1 --no-cpu-baseline --no-kernel-events --no-rollout > $O/ser.log 2>&1 || exit 1
python3 $R/tools/trace_update.py $(ls $O/ser/*/run_kernel_trace.csv $O/ser/run_kernel_trace.csv 2>/dev/null | head -1) --top 30 > $O/ser_breakdown.txt 2>&1
head -25 $O/conc_breakdown.txt; head -25 $O/ser_breakdown.txt
