#!/bin/sh
# r04_ab_cluster.sh TAG LIB... — same-box A/B of libppo builds at C4 and C3, B = 64
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; shift
mkdir -p $O
cd $R
BENCH_ARGS="--config c4 --batch 64 --steps 1 --warmup 1" sh tools/ab_lib.sh "$@" > $O/ab_c4b64.txt 2>&1 || { cat $O/ab_c4b64.txt; exit 1; }
cat $O/ab_c4b64.txt
BENCH_ARGS="--config c3 --batch 64 --steps 2 --warmup 1" sh tools/ab_lib.sh "$@" > $O/ab_c3b64.txt 2>&1 || { cat $O/ab_c3b64.txt; exit 1; }
cat $O/ab_c3b64.txt
