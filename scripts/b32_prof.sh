#!/bin/bash
# b32 step under rocprofv3 (graphed and eager): step span / busy / idle and the top kernels.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/b32prof}; shift
mkdir -p $OUT
export TMPDIR=/tmp
for g in 1 0; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/g$g -o run -- python bench.py --batch 32 --steps 30 --warmup 10 --graph $g "$@" > $OUT/g$g.log 2>&1 || exit $?
  t=$(find $OUT/g$g -name "run_kernel_trace.csv" | head -1)
  echo "== graph $g"; python scripts/step_span.py $t adam_kernel 40
done
