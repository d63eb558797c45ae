#!/bin/sh
# r04_t_ab.sh TAG LIB... — the cluster tests on HEAD, then the per-sub-phase stamp A/B of the given builds
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; shift
mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_cluster.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log; grep "steps vs oracle" $O/tests.log
sh tools/r04_stamps_ab.sh $(basename $O) "$@"
