#!/bin/sh
# r06_ppad2.sh TAG — C4 at B = 64, Pa / Pb partial-slab layouts: row pitch 512 (libppo), slice-major
# [slice][p][b][16] (pslice), pitch 512 + 32 / + 16 (ppad32 / ppad16): stamps of pslice, then update times x2
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
V=$R/ppo.c_amd/lib/variants
PPO_LIB=$V/libppo_pslice.so PPO_CLUSTER_STAMPS=2 timeout -k 10 200 python bench.py --config c4 --batch 64 --steps 1 --warmup 1 \
    --no-cpu-baseline --no-rollout --no-kernel-events > $O/st_pslice.log 2>&1 || exit 1
for i in 1 2; do for v in def pslice ppad32 ppad16; do
  L=$R/ppo.c_amd/lib/libppo.so; [ $v = def ] || L=$V/libppo_$v.so
  PPO_LIB=$L timeout -k 10 200 python bench.py --config c4 --batch 64 --steps 2 --warmup 1 \
      --no-cpu-baseline --no-rollout --no-kernel-events > $O/t_${v}_$i.log 2>&1 || exit 1
done; done
