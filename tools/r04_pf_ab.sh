#!/bin/sh
# r04_pf_ab.sh TAG — the fused value head's rows in flight per wave (4 default / 8 / 2): C4 update A/B
# and a serial trace line of out_head_kernel per build, same box
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
sh tools/ab_lib.sh ppo.c_amd/lib/libppo.so ppo.c_amd/lib/variants/libppo_pf8.so ppo.c_amd/lib/variants/libppo_pf2.so > $O/ab.txt 2>&1 || { cat $O/ab.txt; exit 1; }
cat $O/ab.txt
