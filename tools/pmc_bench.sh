#!/bin/sh
# pmc_bench.sh TAG — the profiles/ evidence for bench.py's roofline (config c4, one timed update):
#   0) rocprofv3 --kernel-trace --stats, production run   → TAG_update_breakdown.txt (value and policy
#      minibatch loops overlapping on two streams: update span vs Σ kernel time)
#   with PPO_SERIAL=1 (loops one after the other, every kernel running alone — the conditions of
#   bench.py's roofline pass):
#   1) rocprofv3 --kernel-trace --stats            → TAG_kernel_stats.csv, TAG_gemm_by_shape.txt
#   2) rocprofv3 --pmc FETCH_SIZE   (own pass, a step-limited sample) ┐ → TAG_pmc_gemm.json: HBM bytes per GEMM launch
#   3) rocprofv3 --pmc WRITE_SIZE   (own pass)      ┘   = (2·FETCH_SIZE + WRITE_SIZE)·1 KiB (gfx950)
# (summarised afterwards on the host with summarize_profile.py / trace_update.py)
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=$1
O=$R/gpurun_out/$T
B="python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-kernel-events --no-rollout"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/conc -o run --output-format csv -- $B > $O.conc.log 2>&1
export PPO_SERIAL=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- $B > $O.trace.log 2>&1
# counter passes serialise every dispatch: a bounded sample of the same launches (32 value + 16
# policy minibatch steps per update, plus GAE's buffer-wide forward)
P="$B --step-limit 32,16"
timeout -k 10 170 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- $P > $O.fetch.log 2>&1
timeout -k 10 170 rocprofv3 --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- $P > $O.write.log 2>&1
