#!/bin/sh
# pmc_x3.sh TAG [OPS] — rocprofv3 counter passes (one pass per line, each its own run) of the x3
# engine at the C4 512x512 shapes (tools/gemm_one.py, GEMM_ENGINE=x3), into gpurun_out/TAG/
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export GEMM_ENGINE=x3
timeout -s KILL 60 rocprofv3 -L > $O/counters_list.txt 2>&1 || true
for op in ${2:-0 1 2}; do
 for pass in "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES" \
             "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU" \
             "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_MFMA" \
             "SQ_INSTS_SALU SQ_INSTS_VMEM SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS" \
             "SQ_VALU_MFMA_COEXEC_CYCLES SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_MFMA_MOPS_BF16" \
             "FETCH_SIZE" "WRITE_SIZE"; do
  tag=$(echo $pass | cut -d' ' -f1)
  timeout -s KILL 60 rocprofv3 --pmc $pass -d $O/op${op}_$tag -o run --output-format csv -- python3 $R/tools/gemm_one.py $op 32768 512 512 -1 20 > $O/op${op}_$tag.log 2>&1 || echo "pass $tag op $op failed" >> $O/failed.txt
 done
done
