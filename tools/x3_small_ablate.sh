#!/bin/sh
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
D=$R/ppo.c_amd/lib/variants/libppo_diag.so
for s in "0 4096 512 512" "1 4096 512 512" "0 8192 256 256"; do
  set -- $s
  n=$3; nk=$((n / 16))
  timeout -k 5 60 python tools/x3_stamps.py --lib $D --op $1 --cfg 4 --nwg $(( ($2/64) * ($4/64) )) --nk $nk $2 $3 $4
  for abl in ${ABLS:-0 1 2 4 8 64}; do
    echo "ablate $abl: $(PPO_LIB=$D PPO_X3_ABLATE=$abl GEMM_ENGINE=x3 timeout -k 5 60 python tools/gemm_one.py $s 4 50)"
  done
done
