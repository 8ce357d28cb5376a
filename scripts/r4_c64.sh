#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/c64
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "c64" > $OUT/kt.log 2>&1
rc=$?; tail -3 $OUT/kt.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench/c64.py > $OUT/c64.log 2>&1; rc=$?; cat $OUT/c64.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --steps 12 --warmup 4 > $OUT/b2560.json 2> $OUT/b2560.err; rc=$?; cat $OUT/b2560.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 env PDDL_C64W=1 python bench.py --steps 12 --warmup 4 > $OUT/b2560w.json 2> $OUT/b2560w.err; rc=$?; cat $OUT/b2560w.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench/stem.py > $OUT/stem.log 2>&1; rc=$?; cat $OUT/stem.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "stem_pool" > $OUT/kt2.log 2>&1; rc=$?; tail -3 $OUT/kt2.log
