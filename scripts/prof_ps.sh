#!/bin/bash
# Kernel trace of the PS entry script on one GPU (1 PS + 1 worker sharing the card) and the
# per-step split of the worker's step span: worker kernels, PS-process kernels, both idle; then
# the single entry script's trace at the same batch and the per-kernel difference.
#   bash scripts/prof_ps.sh OUTDIR [BATCH=32] [STEPS=120]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/prof_ps}; B=${2:-32}; S=${3:-120}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run_%pid% -- \
  python -u imagenet-resnet50-ps.py --ps 1 --worker 1 --data synthetic --epochs 1 --steps-per-epoch $S \
  --validation-steps 0 --batch-size $B --no-save > $OUT/run.log 2>&1 || exit $?
grep -o "[0-9.]* img/s" $OUT/run.log | tail -1
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $OUT/single -o run -- \
  python -u imagenet-resnet50.py --data synthetic --epochs 1 --steps-per-epoch $S \
  --validation-steps 0 --batch-size $B --no-save > $OUT/single.log 2>&1 || exit $?
grep -o "[0-9.]* img/s" $OUT/single.log | tail -1
python scripts/ps_trace.py $(find $OUT/trace -name "*kernel_trace.csv") --ref $(find $OUT/single -name "*kernel_trace.csv")
