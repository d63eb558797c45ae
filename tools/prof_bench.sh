#!/bin/sh
# prof_bench.sh TAG [bench args...] — rocprofv3 kernel trace + stats of one bench update
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
TAG=$1; shift
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/$TAG -o run --output-format csv -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-kernel-events "$@" > $R/gpurun_out/$TAG.log 2>&1
