#!/bin/sh
# r06_c3slice.sh TAG — the B = 64 cluster tests on the slice-major partial slabs, then C3 at B = 64:
# libppo (slice-major G1) vs c3rows (row-major G1), interleaved twice
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_cluster.py -x -v -s --timeout 300 --timeout-method thread > $O/cluster_tests.log 2>&1 || exit 1
V=$R/ppo.c_amd/lib/variants
for i in 1 2; do for v in def c3rows; do
  L=$R/ppo.c_amd/lib/libppo.so; [ $v = def ] || L=$V/libppo_$v.so
  PPO_LIB=$L timeout -k 10 200 python bench.py --config c3 --batch 64 --steps 3 --warmup 1 \
      --no-cpu-baseline --no-rollout --no-kernel-events > $O/c3_${v}_$i.log 2>&1 || exit 1
done; done
