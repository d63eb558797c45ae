#!/bin/sh
# x3_ablate_small.sh TAG — PPO_X3_ABLATE timing ablations (libppo_diag.so) of the x3 forward /
# grad_x at the C4 shape (256x256 tiles) and the G=8 shard shape (64x64 tiles)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
L=$R/ppo.c_amd/lib/variants/libppo_diag.so
for A in 0 64 2 1 8 4; do
  echo "== ABLATE=$A" >> $O/ablate.txt
  PPO_X3_ABLATE=$A PPO_LIB=$L timeout -k 10 120 python3 $R/tools/x3_bench.py --shapes "0,32768,512,512;1,32768,512,512" --cfgs 0 --iters 30 >> $O/ablate.txt || exit 1
  PPO_X3_ABLATE=$A PPO_LIB=$L timeout -k 10 120 python3 $R/tools/x3_bench.py --shapes "0,4096,512,512;1,4096,512,512" --cfgs 4 --iters 50 >> $O/ablate.txt || exit 1
done
