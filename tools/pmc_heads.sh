#!/bin/sh
# pmc_heads.sh TAG — HBM bytes and SQ counters of the output-layer kernels (fused value head,
# A = 17 one-pass backward) in a step-limited C4 update, PPO_SERIAL=1; one rocprofv3 pass per line
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export PPO_SERIAL=1
B="python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-kernel-events --no-rollout --step-limit 8,4"
for pass in "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY" \
            "SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM"; do
  tag=$(echo $pass | cut -d' ' -f1)
  timeout -s KILL 150 rocprofv3 --pmc $pass -d $O/$tag -o run --output-format csv -- $B > $O/$tag.log 2>&1 || { echo "pass $tag failed"; exit 1; }
  echo "pass $tag ok"
done
