#!/bin/sh
# trace_ab.sh TAG VAR "bench args" — serial rocprofv3 kernel traces (PPO_SERIAL=1) of one bench update
# with VAR=0 and VAR=1, each summarised by tools/trace_update.py (gpurun_out/TAG/VAR{0,1}.txt)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
export PPO_SERIAL=1
cd /tmp && export TMPDIR=/tmp
for V in 0 1; do
    export $2=$V
    timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof$V -o run --output-format csv -- python3 $R/bench.py $3 --no-cpu-baseline --no-rollout --no-kernel-events --steps 1 --warmup 1 > $O/prof$V.log 2>&1 || exit 1
    python3 $R/tools/trace_update.py $(find $O/prof$V -name "*kernel_trace.csv" | head -1) --top 24 > $O/$2$V.txt || exit 1
done
