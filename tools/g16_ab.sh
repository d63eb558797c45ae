#!/bin/sh
# g16_ab.sh TAG VARIANT — bf16 forward / grad_x at the C5 shape (gemm16_sweep cfg 9) and the C5 bench line,
# lib/variants/libppo_VARIANT.so (A) against lib/libppo.so (B), A B A B on one box
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
VAR=$R/ppo.c_amd/lib/variants/libppo_$2.so
mkdir -p $O
cd $R
for rep in 1 2; do
  for L in A B; do
    if [ $L = A ]; then export PPO_LIB=$VAR; else unset PPO_LIB; fi
    echo "== $L$rep"
    NO_GRADW=1 timeout -k 5 120 python tools/gemm16_sweep.py --cfgs 9
    timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --no-rollout 2>/dev/null | tail -1 > $O/c5_${L}$rep.json
    python -c "import json; print('c5 ms', round(json.load(open('$O/c5_${L}$rep.json'))['ms_per_step'], 2))"
  done
done
