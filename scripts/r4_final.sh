#!/bin/bash
# Round-4 final check: the whole GPU suite, smoke, the driver's benches, and a per-layer trace of
# the headline step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/final
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $OUT/gputests.log 2>&1
rc=$?; tail -4 $OUT/gputests.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1
rc=$?; tail -1 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
j() { python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1], d['value'], d['ms_per_step'])" $1; }
b() { local tag=$1; shift; timeout -k 10 240 python bench.py "$@" > $OUT/$tag.json 2> $OUT/$tag.err || { echo "$tag failed"; tail -3 $OUT/$tag.err; return 1; }; j $OUT/$tag.json; }
b b2560 --steps 12 --warmup 4 && b b2560b --steps 20 --warmup 5 && b b1024 --batch 1024 --steps 20 --warmup 5 && \
b b32 --batch 32 --steps 40 --warmup 10 && b b32g --batch 32 --steps 40 --warmup 10 --graph 1 && \
b b32c160 --batch 32 --crop 160 --steps 40 --warmup 10 && b b32c160g --batch 32 --crop 160 --steps 40 --warmup 10 --graph 1 && \
b b256c160 --batch 256 --crop 160 --steps 20 --warmup 5 && b fp32 --precision fp32 --steps 10 --warmup 3 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof2560 -o run --output-format csv -- python bench.py --steps 3 --warmup 2 > $OUT/prof2560.log 2>&1
