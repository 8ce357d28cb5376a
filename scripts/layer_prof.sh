#!/bin/bash
# Headline step per-layer trace: bench.py at b2560 under rocprofv3 --kernel-trace, summarised by
# scripts/analyze_trace.py.   bash scripts/layer_prof.sh OUTDIR [bench args...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/layers}; shift
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof -o run -- python bench.py --steps 3 --warmup 2 "$@" > $OUT/prof.log 2>&1 || exit $?
t=$(find $OUT/prof -name "run_kernel_trace.csv" | head -1)
python scripts/analyze_trace.py $t 2560 > $OUT/per_layer.txt 2>&1; tail -12 $OUT/per_layer.txt
