#!/bin/sh
# ab_x3.sh TAG LIB... — x3 parity tests on the current libppo, then x3 launch times at the C4 /
# C4-shard / C3 shapes and a C4 bench line per libppo build (PPO_LIB), interleaved twice
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; shift
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_x3.py tests/test_gpu_ops.py tests/test_gpu_gemm_cfgs.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || exit 1
S=${X3_SHAPES:-"0,32768,512,512;0,32768,376,512;1,32768,512,512;2,32768,512,512;2,32768,376,512;0,4096,512,512;1,4096,512,512;2,4096,512,512"}
for rep in 1 2; do
  for L in "$@"; do
    echo "== $L" >> $O/x3.txt
    PPO_LIB=$L timeout -k 10 120 python3 tools/x3_bench.py --shapes "$S" --iters 50 >> $O/x3.txt || exit 1
    PPO_LIB=$L timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-rollout --no-kernel-events | grep '^{' | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$L', round(d['ms_per_step'],2))" >> $O/bench.txt || exit 1
  done
done
