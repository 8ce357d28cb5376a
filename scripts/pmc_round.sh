#!/bin/bash
# PMC counter passes (one rocprofv3 run per counter group, cdna_hip_programming §profiling) over
# single-kernel probes of representative b1024 layers; summarize with
#   python scripts/pmc_summary.py gpurun_out/pmc
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
P1="SQ_LDS_IDX_ACTIVE SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL"
P2="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_MFMA"
P3="SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_INST_LEVEL_LDS"
run() {  # tag op shape
  local i=0
  for P in "$P1" "$P2" "$P3"; do
    i=$((i + 1))
    timeout -s KILL 90 rocprofv3 --pmc $P -d gpurun_out/pmc/pmc_$1_$i -o run --output-format csv -- \
      python scripts/kprobe.py --op $2 --shape $3 --iters 10 > gpurun_out/pmc/$1_$i.log 2>&1 || return 1
  done
}
run fwd_s3 fwd 1024,28,128,128,3,1,1 && run fwd_s4 fwd 1024,14,256,256,3,1,1 && \
run fwd_s5 fwd 1024,7,512,512,3,1,1 && run fwd_s2 fwd 1024,56,64,64,3,1,1 && \
run wg_s3 wgrad 1024,28,128,128,3,1,1 && run wg_s4 wgrad 1024,14,256,256,3,1,1 && \
run dg_s4c1 dgrad_add 1024,14,1024,256,1,1,0 && \
run fwdres_s3c3 fwdres 1024,28,128,512,1,1,0 && run fwdres_s4c3 fwdres 1024,14,256,1024,1,1,0
