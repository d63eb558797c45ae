#!/bin/sh
# r06_n2_onegpu.sh TAG — a world-size-2 rehearsal of the data-parallel bench on ONE GPU: two ranks (RANK 0/1,
# LOCAL_RANK 0 for both) with real RCCL communicators (the per-loop split, inline all-reduces, replica check).
# Both ranks are children of one shell (bench.py names the RCCL unique-id file after the parent pid).
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
run2() {  # name, bench args...
  n=$1; shift
  timeout -k 10 240 sh -c "
    RANK=0 WORLD_SIZE=2 LOCAL_RANK=0 NCCL_DEBUG=WARN python bench.py --gpus 2 $* > $O/${n}_r0.log 2>&1 &
    RANK=1 WORLD_SIZE=2 LOCAL_RANK=0 NCCL_DEBUG=WARN python bench.py --gpus 2 $* > $O/${n}_r1.log 2>&1 &
    wait %1; r0=\$?; wait %2; r1=\$?; echo \"$n rc \$r0 \$r1\" >> $O/rc.txt; [ \$r0 -eq 0 ] && [ \$r1 -eq 0 ]"
}
run2 c4 --steps 2 --warmup 1 --no-cpu-baseline --no-rollout || exit 1
PPO_COMM_ASYNC=1 run2 c4async --steps 2 --warmup 1 --no-cpu-baseline --no-rollout || exit 1
