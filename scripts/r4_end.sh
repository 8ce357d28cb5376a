#!/bin/bash
# End-of-round check of the tree as committed (rebuilt in a fresh container): the GPU suite, smoke
# and the driver's headline benches.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/end
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $OUT/gputests.log 2>&1
rc=$?; tail -3 $OUT/gputests.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?; tail -1 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
j() { python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1], d['value'], d['ms_per_step'])" $1; }
b() { local tag=$1; shift; timeout -k 10 240 python bench.py "$@" > $OUT/$tag.json 2> $OUT/$tag.err || { echo "$tag failed"; tail -3 $OUT/$tag.err; return 1; }; j $OUT/$tag.json; }
b b2560 --steps 12 --warmup 4 && b b2560b --steps 20 --warmup 5 && b b1024 --batch 1024 --steps 20 --warmup 5 && \
b b32g --batch 32 --steps 40 --warmup 10 --graph 1 && b fp32 --precision fp32 --steps 10 --warmup 3
