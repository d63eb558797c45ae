#!/bin/sh
# trace_config.sh TAG "bench args" — rocprofv3 kernel traces of one bench update of HEAD, serial
# (PPO_SERIAL=1) and concurrent, each summarised by tools/trace_update.py (gpurun_out/TAG/{serial,conc}.txt)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for M in serial conc; do
    if [ $M = serial ]; then export PPO_SERIAL=1; else unset PPO_SERIAL; fi
    timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof_$M -o run --output-format csv -- python3 $R/bench.py $2 --no-cpu-baseline --no-rollout --no-kernel-events --steps 1 --warmup 1 > $O/prof_$M.log 2>&1 || exit 1
    python3 $R/tools/trace_update.py $(find $O/prof_$M -name "*kernel_trace.csv" | head -1) --top 30 > $O/$M.txt || exit 1
done
