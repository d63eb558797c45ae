#!/bin/sh
# r06_b64diag.sh TAG — C4 at B = 64 with every workgroup's barrier arrival / exit stamped (PPO_CLUSTER_STAMPS=2,
# 4 updates), then a PMC pass of address-translation and stall counters per dispatch; and the C4 copy-store A/B
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
PPO_CLUSTER_STAMPS=2 timeout -k 10 200 python bench.py --config c4 --batch 64 --steps 3 --warmup 1 --no-cpu-baseline --no-rollout --no-kernel-events > $O/c4b64_arrivals.log 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 240 python bench.py --no-cpu-baseline --no-rollout > $O/c4_$i.log 2>&1 || exit 1
  PPO_LIB=$R/ppo.c_amd/lib/variants/libppo_copynt.so timeout -k 10 240 python bench.py --no-cpu-baseline --no-rollout > $O/c4_copynt_$i.log 2>&1 || exit 1
done
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_REQUEST_sum TCP_TCR_TCP_STALL_CYCLES_sum \
    TCP_UTCL1_SERIALIZATION_STALL_sum TCC_TAG_STALL_sum -d $O/pmc2 -o b64 --output-format csv -- \
    python3 $R/bench.py --config c4 --batch 64 --steps 3 --warmup 1 --no-cpu-baseline --no-rollout --no-kernel-events \
    > $O/pmc2_b64.log 2>&1
