#!/bin/sh
# r04_ab_x3.sh TAG — x3 launch times at the C4 shapes and the C4 bench, HEAD vs lib/variants/libppo_base.so
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
SH="0,32768,512,512;0,32768,376,512;1,32768,512,512;2,32768,512,512;2,32768,376,512;0,4096,512,512;2,4096,512,512"
PPO_LIB=ppo.c_amd/lib/libppo.so timeout -k 10 200 python3 tools/x3_bench.py --shapes "0,32768,512,512;1,32768,512,512;0,32768,376,512" --cfgs 0,1,2 --iters 50 > $O/x3cfg.txt 2>&1 || exit 1
for L in ppo.c_amd/lib/libppo.so ppo.c_amd/lib/variants/libppo_base.so ppo.c_amd/lib/libppo.so ppo.c_amd/lib/variants/libppo_base.so; do
  echo "== $L" >> $O/x3.txt
  PPO_LIB=$L timeout -k 10 120 python3 tools/x3_bench.py --shapes "$SH" --iters 50 >> $O/x3.txt 2>&1 || exit 1
done
sh tools/ab_bench.sh $1 "--steps 5 --warmup 2" ppo.c_amd/lib/libppo.so ppo.c_amd/lib/variants/libppo_base.so
for L in diag basediag; do
  for a in "--op 2 --cfg 3 --nwg 256 --nk 64 32768 512 512" "--op 0 32768 512 512" "--op 0 32768 376 512"; do
    echo "== $L $a" >> $O/stamps.txt
    timeout -k 10 120 python3 tools/x3_stamps.py --lib ppo.c_amd/lib/variants/libppo_$L.so $a >> $O/stamps.txt 2>&1 || exit 1
  done
done
