#!/bin/bash
# Packed ReLU-bit stores: kernel tests, per-layer A/B (4-byte vs 1-byte stores), b2560 bench,
# kernel trace, GPU suite, smoke.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/bits2
mkdir -p $OUT
export TMPDIR=/tmp
j() { python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1], d['value'], d['ms_per_step'])" $1; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -v -x --timeout 120 --timeout-method thread -k "bits or bitmask or pk_matches" > $OUT/kt.log 2>&1
rc=$?; grep -E "FAIL|^E |passed|failed" $OUT/kt.log | head -20; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench/bits_ab.py > $OUT/ab.txt 2>&1; rc=$?; cat $OUT/ab.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --steps 12 --warmup 4 > $OUT/b1.json 2> $OUT/b1.err; rc=$?; j $OUT/b1.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $OUT/b2.json 2> $OUT/b2.err; rc=$?; j $OUT/b2.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof2560 -o run --output-format csv -- python bench.py --steps 3 --warmup 2 > $OUT/prof2560.log 2>&1 || exit $?
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $OUT/gputests.log 2>&1
rc=$?; tail -3 $OUT/gputests.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?; tail -1 $OUT/smoke.log; exit $rc
