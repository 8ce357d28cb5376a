#!/bin/bash
# Kernel traces of the single and Mirrored entry scripts (the presets' crop 244) and the per-step
# span / busy / idle summary of each: single, Mirrored on one GPU (one replica: the eager step)
# and Mirrored forced onto the multi-replica schedule (PDDL_MIRROR=segmented=1: segmented HIP
# graphs + grouped bucket all-reduce, what 2-8 replicas run).
#   bash scripts/prof_strategies.sh OUTDIR [BATCH=256]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/profstrat}
BATCH=${2:-256}
mkdir -p $OUT
export TMPDIR=/tmp
C="--data synthetic --epochs 1 --steps-per-epoch 14 --validation-steps 0 --batch-size $BATCH --no-save"
for s in single mirror mirrorseg; do
  f=imagenet-resnet50.py; [ $s != single ] && f=imagenet-resnet50-mirror.py
  seg=0; [ $s = mirrorseg ] && seg=1
  PDDL_MIRROR=segmented=$seg timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/$s -o run -- \
    python $f $C > $OUT/$s.log 2>&1 || exit $?
  t=$(find $OUT/$s -name "run_kernel_trace.csv" | head -1)
  echo "== $s b$BATCH: $(grep -o "[0-9.]* img/s" $OUT/$s.log | tail -1)"; python scripts/step_span.py $t adam_kernel 25; rm -rf $OUT/$s
done
