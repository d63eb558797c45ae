#!/bin/sh
# r04_tol_report.sh TAG — every GPU test with the GEMM-tolerance margins logged (err / tol per check)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
rm -f $O/tol.tsv
PPO_TOL_REPORT=$O/tol.tsv timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/ > $O/test.log 2>&1
tail -1 $O/test.log
sort -rn $O/tol.tsv | head -12
wc -l < $O/tol.tsv
