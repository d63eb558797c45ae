#!/bin/sh
# pmc_c4b64.sh TAG — C4 at B = 64 (cluster_deep phases): per-dispatch memory-side latency counters beside the
# dispatch durations, to tell the fast and slow barrier modes apart (average EA read latency =
# TCC_EA0_RDREQ_LEVEL / TCC_EA0_RDREQ; L1 -> L2 read latency = TCP_TCC_READ_REQ_LATENCY / TCP_TCC_READ_REQ)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_LEVEL_sum TCC_HIT_sum TCC_MISS_sum \
    TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum -d $O/pmc -o b64 --output-format csv -- \
    python3 $R/bench.py --config c4 --batch 64 --steps 5 --warmup 1 --no-cpu-baseline --no-rollout --no-kernel-events \
    > $O/pmc_b64.log 2>&1
