#!/bin/bash
# Kernel trace of the Horovod preset (b32, crop 160) through the Trainer with the segmented
# multi-rank schedule over a 1-rank RCCL communicator (PDDL_COMM=graphs) and the whole-step graph.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/hvdprof}; shift
mkdir -p $OUT
export TMPDIR=/tmp
H="--data synthetic --epochs 1 --steps-per-epoch 40 --validation-steps 0 --batch-size 32 --no-save"
for mode in graphs whole; do
  if [ $mode = graphs ]; then export PDDL_COMM=graphs; X=""; else unset PDDL_COMM; X="--graphs"; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/$mode -o run -- python imagenet-resnet50-hvd.py $H $X "$@" > $OUT/$mode.log 2>&1 || exit $?
  t=$(find $OUT/$mode -name "run_kernel_trace.csv" | head -1)
  echo "== $mode"; python scripts/step_span.py $t adam_kernel 12
done
