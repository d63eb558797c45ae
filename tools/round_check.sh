#!/bin/sh
# round_check.sh TAG — the round-end evidence on one GPU box: the -m gpu suite, smoke(), the default
# bench line, and rocprofv3 --kernel-trace --stats of the same bench command (gpurun_out/TAG/)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
echo "pytest rc=$?" >> $O/gputest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 240 python bench.py > $O/bench.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline > $O/prof.log 2>&1
