#!/bin/sh
# r04_final_a.sh TAG — round-end check part 1: every GPU test (one pytest process), smoke(), the
# default bench line, and a serial (PPO_SERIAL=1) rocprofv3 kernel trace of one C4 update of HEAD
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print('bench', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['dominant']['template'])"
sh tools/r04_serial_trace.sh $1/trace || exit 1
head -8 $O/trace/breakdown.txt
