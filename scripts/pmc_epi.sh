#!/bin/bash
# PMC passes over the epilogue-bound short-K 1x1 layers (the conv3 forwards with the residual,
# the conv1 data gradients with the residual-gradient add) at b1024; summarize with
#   python scripts/pmc_summary.py gpurun_out/pmce
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${1:-gpurun_out/pmce}
mkdir -p $OUT
P1="SQ_LDS_IDX_ACTIVE SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL"
P2="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_MFMA"
P3="SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_INST_LEVEL_LDS"
run() {  # tag op shape
  local i=0
  for P in "$P1" "$P2" "$P3"; do
    i=$((i + 1))
    timeout -s KILL 90 rocprofv3 --pmc $P -d $OUT/pmc_$1_$i -o run --output-format csv -- \
      python scripts/kprobe.py --op $2 --shape $3 --iters 10 > $OUT/$1_$i.log 2>&1 || return 1
  done
}
run fwdres_s3c3 fwdres 1024,28,128,512,1,1,0 && run fwdres_s4c3 fwdres 1024,14,256,1024,1,1,0 && \
run dg_s3c1 dgrad_add 1024,28,512,128,1,1,0 && run dg_s4c1 dgrad_add 1024,14,1024,256,1,1,0 && \
python scripts/pmc_summary.py $OUT
