#!/bin/bash
# Kernel traces of the single and Mirrored entry scripts at b256 / crop 244 (the reference's
# crop, presets' strategies) and the per-step span / busy / idle summary of each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/profstrat}
BATCH=${2:-256}
mkdir -p $OUT
export TMPDIR=/tmp
C="--data synthetic --epochs 1 --steps-per-epoch 14 --validation-steps 0 --batch-size $BATCH --no-save"
for s in single mirror; do
  f=imagenet-resnet50.py; [ $s = mirror ] && f=imagenet-resnet50-mirror.py
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/$s -o run -- python $f $C > $OUT/$s.log 2>&1 || exit $?
  t=$(find $OUT/$s -name "run_kernel_trace.csv" | head -1)
  echo "== $s b$BATCH"; python scripts/step_span.py $t stem_s2d 14
done
