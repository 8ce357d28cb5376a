#!/bin/bash
# Measured-bytes roofline of the headline step: a kernel trace plus one counter pass per byte
# counter over the same short bench.py run, joined by scripts/roofline.py.
#   bash scripts/roofline.sh OUTDIR [bench args...]     (BATCH / CROP env for the analyzer)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/roof}; shift
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run -- \
  python bench.py --steps 2 --warmup 1 "$@" > $OUT/trace.log 2>&1 || exit $?
for P in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $P --output-format csv -d $OUT/$P -o run -- \
    python bench.py --steps 2 --warmup 1 "$@" > $OUT/$P.log 2>&1 || exit $?
done
t=$(find $OUT/trace -name "run_kernel_trace.csv" | head -1)
f=$(find $OUT/FETCH_SIZE -name "run_counter_collection.csv" | head -1)
w=$(find $OUT/WRITE_SIZE -name "run_counter_collection.csv" | head -1)
python scripts/roofline.py $t $f $w ${BATCH:-2560} ${CROP:-224} > $OUT/roofline.txt 2>&1; tail -30 $OUT/roofline.txt
