#!/bin/sh
# r06_check.sh TAG — round-6 GPU pass: the comm / replica tests and the chaos-floor margins verbosely,
# then the whole -m gpu suite, then C4 A/B lines (default, PPO_X3_PAIR=0, PPO_X0_COPY=1, default again),
# the G = 8 shard (one-rank RCCL, inline and PPO_COMM_ASYNC=1), the small-shape engine comparison and
# the C4 B = 64 shader-clock stamps into gpurun_out/TAG/
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_comm.py "tests/test_gpu_update.py::test_comm_rehearsal" -x -v \
    --timeout 120 --timeout-method thread > $O/comm_tests.log 2>&1 || exit 1
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 || exit 1
timeout -k 10 240 python bench.py --no-cpu-baseline > $O/c4.log 2>&1 || exit 1
PPO_X3_PAIR=0 timeout -k 10 240 python bench.py --no-cpu-baseline --no-rollout > $O/c4_nopair.log 2>&1 || exit 1
PPO_X0_COPY=1 timeout -k 10 240 python bench.py --no-cpu-baseline --no-rollout > $O/c4_x0copy.log 2>&1 || exit 1
timeout -k 10 240 python bench.py --no-cpu-baseline --no-rollout > $O/c4_b.log 2>&1 || exit 1
PPO_COMM_SELF=1 timeout -k 10 240 python bench.py --emulate-world 8 --no-cpu-baseline --no-rollout > $O/shard8.log 2>&1 || exit 1
PPO_COMM_SELF=1 PPO_COMM_ASYNC=1 timeout -k 10 240 python bench.py --emulate-world 8 --no-cpu-baseline --no-rollout > $O/shard8_async.log 2>&1 || exit 1
timeout -k 10 120 python tools/engine_small_shapes.py > $O/engines.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_cluster.py -x -v -s -k "chaos_floor or full_update" \
    --timeout 300 --timeout-method thread > $O/chaos.log 2>&1 || exit 1
PPO_CLUSTER_STAMPS=1 timeout -k 10 200 python bench.py --config c4 --batch 64 --steps 3 --warmup 1 --no-cpu-baseline --no-rollout --no-kernel-events > $O/c4b64_clock.log 2>&1 || exit 1
