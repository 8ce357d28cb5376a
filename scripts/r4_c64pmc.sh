#!/bin/bash
# counter passes over the 64-channel 3x3 kernels (bench/c64.py), one pass per counter group
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/c64pmc
mkdir -p $OUT
export TMPDIR=/tmp
i=0
while read -r line; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $line -d $OUT/pmc_$i -o run --output-format csv -- python bench/c64.py --iters 3 > $OUT/pmc_$i.log 2>&1 || exit 1
done <<'PM'
SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT
SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_MFMA
SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_INST_LEVEL_LDS SQ_INSTS_VMEM
PM
python scripts/pmc_summary.py $OUT > $OUT/summary.txt 2>&1; cat $OUT/summary.txt
