#!/bin/sh
# r04_tests.sh TAG [pytest args...] — the given GPU tests, one pytest process, bounded
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; shift
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu "$@" > $O/test.log 2>&1
echo "pytest rc=$?" >> $O/test.log
tail -3 $O/test.log
