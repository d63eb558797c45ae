#!/bin/sh
# r06_lds_abl.sh TAG — x3 at C4's 32768x512x512 (diag build, results wrong): the cost of the LDS fragment reads —
# PPO_X3_ABLATE 256 (no B fragment reads after the prologue), 512 (no A), 768 (neither) — for grad_W (op 2),
# forward (op 0) and grad_x (op 1), beside the production kernel (0)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
D=$R/ppo.c_amd/lib/variants/libppo_diag.so
for op in 2 0 1; do for abl in 0 256 512 768 2; do
  echo "op $op ablate $abl: $(PPO_LIB=$D PPO_X3_ABLATE=$abl GEMM_ENGINE=x3 timeout -k 5 60 python tools/gemm_one.py $op 32768 512 512 -1 30)" >> $O/abl.txt || exit 1
done; done
