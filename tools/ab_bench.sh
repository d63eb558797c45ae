#!/bin/sh
# ab_bench.sh TAG VARIANT [CONFIGS] — bench.py lines of lib/variants/libppo_VARIANT.so (A) and lib/libppo.so
# (B), run A B A B per config so box drift shows (configs: shard8 = rank 0 of a G = 8 split, or any
# --config name; default "shard8 c3 c4").  Output under gpurun_out/TAG/.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
VAR=$R/ppo.c_amd/lib/variants/libppo_$2.so
mkdir -p $O
cd $R
for rep in 1 2; do
  for cfg in ${3:-shard8 c3 c4}; do
    for L in A B; do
      if [ $L = A ]; then export PPO_LIB=$VAR; else unset PPO_LIB; fi
      if [ $cfg = shard8 ]; then
        PPO_COMM_SELF=1 timeout -k 10 300 python bench.py --emulate-world 8 --no-cpu-baseline --no-rollout 2>/dev/null | tail -1 > $O/${cfg}_${L}$rep.json
      else
        timeout -k 10 300 python bench.py --config $cfg --no-cpu-baseline --no-rollout 2>/dev/null | tail -1 > $O/${cfg}_${L}$rep.json
      fi
    done
  done
done
unset PPO_LIB
for f in $O/*.json; do python -c "import json; d=json.load(open('$f')); print('$f'.split('/')[-1], round(d['ms_per_step'], 2))"; done
