#!/bin/bash
# End-to-end check on one GPU: the whole GPU suite, smoke, the driver's benches and a per-layer
# kernel trace of the headline step.   bash scripts/gpu_check.sh [OUTDIR=gpurun_out/check] [quick]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/check}
MODE=${2:-full}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $OUT/gputests.log 2>&1
rc=$?; tail -4 $OUT/gputests.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1
rc=$?; tail -1 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
j() { python -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]);print(sys.argv[1], d['value'], d['ms_per_step'])" $1; }
b() { local tag=$1; shift; timeout -k 10 240 python bench.py "$@" > $OUT/$tag.json 2> $OUT/$tag.err || { echo "$tag failed"; tail -3 $OUT/$tag.err; return 1; }; j $OUT/$tag.json; }
b b2560 --steps 20 --warmup 5 || exit 1
[ "$MODE" = quick ] && exit 0
b b1024 --batch 1024 --steps 20 --warmup 5 && b b256 --batch 256 --steps 30 --warmup 5 && \
b b256c160 --batch 256 --crop 160 --steps 30 --warmup 5 && \
b b32 --batch 32 --steps 40 --warmup 10 && b b32g --batch 32 --steps 40 --warmup 10 --graph 1 && \
b b32c160g --batch 32 --crop 160 --steps 40 --warmup 10 --graph 1 && \
b fp32 --precision fp32 --steps 10 --warmup 3 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof2560 -o run --output-format csv -- python bench.py --steps 3 --warmup 2 > $OUT/prof2560.log 2>&1
