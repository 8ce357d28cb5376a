#!/bin/bash
# Round 4: 64-channel 3x3 conv kernels (row tiles vs pixel ring) and the fused-stem variants:
# numerics, per-kernel A/B, end-to-end b2560.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/c64
mkdir -p $OUT
export TMPDIR=/tmp
j() { python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1], d['value'], d['ms_per_step'])" $1; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "c64 or stem_pool" > $OUT/kt.log 2>&1
rc=$?; tail -3 $OUT/kt.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench/c64.py > $OUT/c64.log 2>&1; rc=$?; cat $OUT/c64.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 env PDDL_KNOBS=c64=1 python bench/c64.py > $OUT/c64ring.log 2>&1; rc=$?; grep -E "_ring" $OUT/c64ring.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench/stem.py > $OUT/stem.log 2>&1; rc=$?; cat $OUT/stem.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --steps 12 --warmup 4 > $OUT/b2560.json 2> $OUT/b2560.err; rc=$?; j $OUT/b2560.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 env PDDL_KNOBS=c64=1 python bench.py --steps 12 --warmup 4 > $OUT/b2560ring.json 2> $OUT/b2560ring.err; rc=$?; j $OUT/b2560ring.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 env PDDL_KNOBS=stem_pool=0 python bench.py --steps 12 --warmup 4 > $OUT/b2560stem0.json 2> $OUT/b2560stem0.err; rc=$?; j $OUT/b2560stem0.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof2560 -o run --output-format csv -- python bench.py --steps 3 --warmup 2 > $OUT/prof2560.log 2>&1
