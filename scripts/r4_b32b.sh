#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/b32b
mkdir -p $OUT
export TMPDIR=/tmp
j() { python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1], d['value'], d['ms_per_step'])" $1; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -x --timeout 120 --timeout-method thread -k "stem_pool" > $OUT/kt.log 2>&1
rc=$?; tail -2 $OUT/kt.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -q -x --timeout 200 --timeout-method thread -k "reference or two_stream or graphed" > $OUT/eng.log 2>&1
rc=$?; tail -2 $OUT/eng.log; [ $rc -eq 0 ] || exit $rc
for t in a b; do
timeout -k 10 200 python bench.py --batch 32 --steps 60 --warmup 10 > $OUT/b32$t.json 2> $OUT/b32.err; rc=$?; j $OUT/b32$t.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --batch 32 --steps 60 --warmup 10 --graph 1 > $OUT/b32g$t.json 2> $OUT/b32g.err; rc=$?; j $OUT/b32g$t.json; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 200 python bench.py --batch 32 --crop 160 --steps 60 --warmup 10 > $OUT/b32c160.json 2> $OUT/b32c.err; rc=$?; j $OUT/b32c160.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --batch 32 --crop 160 --steps 60 --warmup 10 --graph 1 > $OUT/b32c160g.json 2> $OUT/b32cg.err; rc=$?; j $OUT/b32c160g.json
