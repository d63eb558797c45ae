#!/bin/sh
# r04_c5_trace.sh TAG — serial rocprofv3 kernel trace of one C5 update (bf16)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
PPO_SERIAL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/ser -o run --output-format csv -- python3 $R/bench.py --config c5 --steps 1 --warmup 1 --no-cpu-baseline --no-kernel-events --no-rollout > $O/ser.log 2>&1 || exit 1
python3 $R/tools/trace_update.py $(ls $O/ser/*/run_kernel_trace.csv $O/ser/run_kernel_trace.csv 2>/dev/null | head -1) --top 30 > $O/ser_breakdown.txt 2>&1
head -24 $O/ser_breakdown.txt
