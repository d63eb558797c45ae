#!/bin/sh
# trace_libs.sh TAG VARIANT "bench args" — serial rocprofv3 kernel traces (PPO_SERIAL=1) of one bench
# update with lib/variants/libppo_VARIANT.so (A) and lib/libppo.so (B), each summarised by
# tools/trace_update.py (gpurun_out/TAG/{A,B}.txt)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
export PPO_SERIAL=1
cd /tmp && export TMPDIR=/tmp
for L in A B; do
    if [ $L = A ]; then export PPO_LIB=$R/ppo.c_amd/lib/variants/libppo_$2.so; else unset PPO_LIB; fi
    timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof$L -o run --output-format csv -- python3 $R/bench.py $3 --no-cpu-baseline --no-rollout --no-kernel-events --steps 1 --warmup 1 > $O/prof$L.log 2>&1 || exit 1
    python3 $R/tools/trace_update.py $(find $O/prof$L -name "*kernel_trace.csv" | head -1) --top 24 > $O/$L.txt || exit 1
done
