#!/bin/sh
# ab_variants.sh V1 V2 ... — x3 launch times at the C4 shapes and a C4 bench line per libppo variant
# (ppo.c_amd/lib/variants/libppo_V.so; "base" = ppo.c_amd/lib/libppo.so), interleaved twice
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/ab
mkdir -p $O
for rep in 1 2; do
  for v in "$@"; do
    if [ "$v" = base ]; then L=$R/ppo.c_amd/lib/libppo.so; else L=$R/ppo.c_amd/lib/variants/libppo_$v.so; fi
    PPO_LIB=$L timeout -k 10 120 python3 $R/tools/x3_bench.py --shapes "0,32768,512,512;1,32768,512,512;2,32768,512,512" --iters 50 | sed "s/^/$v /" >> $O/x3.txt || exit 1
    PPO_LIB=$L timeout -k 10 120 python3 $R/bench.py --no-cpu-baseline --no-rollout --no-kernel-events | grep '^{' | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', round(d['ms_per_step'],2))" >> $O/bench.txt || exit 1
  done
done
