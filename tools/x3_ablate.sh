#!/bin/sh
# x3_ablate.sh — time the x3 forward (C4 512x512, cfg 0) with parts of the kernel removed (PPO_X3_ABLATE),
# then SQ counter passes of the production kernel (one rocprofv3 pass per line)
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/x3abl
mkdir -p $O
export PPO_LIB=${PPO_LIB:-$R/ppo.c_amd/lib/variants/libppo_diag.so}   # tools/build_variant.sh diag -DPPO_X3_DIAG gemm_x3
for ab in 0 1 2 4 8; do
  PPO_X3_ABLATE=$ab GEMM_ENGINE=x3 timeout -k 10 60 python3 $R/tools/gemm_one.py ${OP:-0} 32768 512 512 0 50 | sed "s/^/ablate=$ab /" >> $O/times.txt || exit 1
done
cd /tmp && export TMPDIR=/tmp
for pass in "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU" "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_MFMA" "SQ_INSTS_SALU SQ_INSTS_VMEM SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS"; do
  tag=$(echo $pass | cut -d' ' -f1)
  GEMM_ENGINE=x3 timeout -k 10 120 rocprofv3 --pmc $pass -d $O/$tag -o run --output-format csv -- python3 $R/tools/gemm_one.py ${OP:-0} 32768 512 512 0 20 > $O/$tag.log 2>&1 || exit 1
done
