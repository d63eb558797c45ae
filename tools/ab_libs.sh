#!/bin/sh
# ab_libs.sh TAG VARIANT — one-box A/B of lib/variants/libppo_VARIANT.so (A) against lib/libppo.so (B):
# x3 GEMM timings at the shard / C3 / C4 shapes, then bench.py lines (G = 8 shard, C3, C4) run A B A B so
# box drift shows.  Output under gpurun_out/TAG/.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
VAR=$R/ppo.c_amd/lib/variants/libppo_$2.so
mkdir -p $O
cd $R
gemms() {
    for s in "0 4096 512 512" "1 4096 512 512" "2 4096 512 512" "0 4096 376 512" "2 4096 376 512" \
             "0 8192 256 256" "1 8192 256 256" "2 8192 256 256" "0 32768 512 512" "1 32768 512 512" "2 32768 512 512"; do
        GEMM_ENGINE=x3 timeout -k 5 60 python tools/gemm_one.py $s -1 50
    done
}
echo "== A ($2)" > $O/gemm.txt
PPO_LIB=$VAR gemms >> $O/gemm.txt
echo "== B (lib/libppo.so)" >> $O/gemm.txt
gemms >> $O/gemm.txt
for rep in 1 2; do
    for L in A B; do
        if [ $L = A ]; then export PPO_LIB=$VAR; else unset PPO_LIB; fi
        PPO_COMM_SELF=1 timeout -k 10 200 python bench.py --emulate-world 8 --no-cpu-baseline --no-rollout 2>/dev/null | tail -1 > $O/shard8_${L}$rep.json
        timeout -k 10 200 python bench.py --config c3 --no-cpu-baseline --no-rollout 2>/dev/null | tail -1 > $O/c3_${L}$rep.json
        timeout -k 10 200 python bench.py --no-cpu-baseline --no-rollout 2>/dev/null | tail -1 > $O/c4_${L}$rep.json
    done
done
unset PPO_LIB
python - "$O" <<'EOF'
import json, sys, glob, os
o = sys.argv[1]
for f in sorted(glob.glob(os.path.join(o, "*.json"))):
    try:
        d = json.load(open(f))
        print(f"{os.path.basename(f):16s} {d['ms_per_step']:8.2f} ms")
    except Exception as e:
        print(f, "unreadable", e)
EOF
