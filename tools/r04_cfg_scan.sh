#!/bin/sh
# r04_cfg_scan.sh TAG — x3 tile configurations at the C4 and G = 8 shard shapes
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
timeout -k 10 300 python3 tools/x3_bench.py --shapes "0,32768,512,512;1,32768,512,512;0,32768,376,512;2,32768,512,512" --cfgs 0,5 --iters 50 > $O/cfg_c4.txt 2>&1 || exit 1
timeout -k 10 300 python3 tools/x3_bench.py --shapes "0,4096,512,512;1,4096,512,512;0,4096,376,512;2,4096,512,512;2,4096,376,512" --cfgs 1,2,4,5,3 --iters 100 > $O/cfg_shard.txt 2>&1 || exit 1
