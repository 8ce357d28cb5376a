# ad-hoc GPU session: PMC counter passes (one rocprofv3 run per counter group) over the fused
# conv3 backward kernels at the b1024 stage-2 / stage-3 shapes; summarize with
#   python scripts/pmc_summary.py gpurun_out/pmc
set -o pipefail
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
P1="SQ_LDS_IDX_ACTIVE SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL"
P2="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_MFMA"
P3="SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_INST_LEVEL_LDS"
P4="FETCH_SIZE"
P5="WRITE_SIZE"
run() {  # tag op shape
  local i=0
  for P in "$P1" "$P2" "$P3" "$P4" "$P5"; do
    i=$((i + 1))
    timeout -s KILL 90 rocprofv3 --pmc $P -d gpurun_out/pmc/pmc_$1_$i -o run --output-format csv -- \
      python scripts/kprobe.py --op $2 --shape $3 --iters 10 > gpurun_out/pmc/$1_$i.log 2>&1 || return 1
  done
}
timeout -k 10 120 python scripts/kprobe.py --op bwd1x1 --shape 1024,56,64,256,1,1,0 --iters 20 > gpurun_out/pmc/t2.log 2>&1 && \
timeout -k 10 120 python scripts/kprobe.py --op bwd1x1 --shape 1024,28,128,512,1,1,0 --iters 20 > gpurun_out/pmc/t3.log 2>&1 && \
run b1_s2 bwd1x1 1024,56,64,256,1,1,0 && run b1_s3 bwd1x1 1024,28,128,512,1,1,0
rc=$?
cat gpurun_out/pmc/t2.log gpurun_out/pmc/t3.log | grep '"op"'
exit $rc
