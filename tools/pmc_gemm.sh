# pmc_gemm.sh [OPS] — SQ/GRBM counter passes (one pass per line) of gemm_one.py at the C4 512x512 shape
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc
for op in ${1:-0 2}; do
 for pass in "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU" "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_MFMA" "SQ_INSTS_SALU SQ_INSTS_VMEM SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS"; do
  tag=$(echo $pass | cut -d' ' -f1)
  timeout -k 10 120 rocprofv3 --pmc $pass -d $R/gpurun_out/pmc/op${op}_$tag -o run --output-format csv -- python3 $R/tools/gemm_one.py $op 32768 512 512 -1 20 > $R/gpurun_out/pmc/op${op}_$tag.log 2>&1
 done
done
