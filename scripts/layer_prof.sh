#!/bin/bash
# Per-layer trace of a training step: bench.py under rocprofv3 --kernel-trace, summarised by
# scripts/analyze_trace.py.   bash scripts/layer_prof.sh OUTDIR [bench args...]
# (BATCH=256 CROP=224 for other configs; use PDDL_ENGINE=two_stream=0 below b1024 so the launch order
# matches the analyzer's single-stream schedule)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/layers}; shift
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof -o run -- python bench.py --steps 3 --warmup 2 "$@" > $OUT/prof.log 2>&1 || exit $?
t=$(find $OUT/prof -name "run_kernel_trace.csv" | head -1)
python scripts/analyze_trace.py $t ${BATCH:-2560} ${CROP:-224} "$PDDL_KNOBS" > $OUT/per_layer.txt 2>&1; tail -12 $OUT/per_layer.txt
