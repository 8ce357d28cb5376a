#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/pre
mkdir -p $OUT
export TMPDIR=/tmp
j() { python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1], d['value'], d['ms_per_step'])" $1; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -v -x --timeout 120 --timeout-method thread -k "bwd1x1" > $OUT/kt.log 2>&1
rc=$?; grep -E "PASS|FAIL|^E " $OUT/kt.log | head -20; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -v -s --timeout 200 --timeout-method thread -k "c1_dgrad_fused or two_stream or graphed_step" > $OUT/eng.log 2>&1
rc=$?; grep -E "PASS|FAIL|^E |c1pre:|ratio" $OUT/eng.log | head -20; [ $rc -le 1 ] || exit $rc
timeout -k 10 200 python bench.py --steps 12 --warmup 4 > $OUT/b2560.json 2> $OUT/b2560.err; rc=$?; j $OUT/b2560.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 env PDDL_C1PRE=0 python bench.py --steps 12 --warmup 4 > $OUT/b2560off.json 2> $OUT/b2560off.err; rc=$?; j $OUT/b2560off.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --batch 32 --steps 60 --warmup 10 --graph 1 > $OUT/b32g.json 2> $OUT/b32g.err; rc=$?; j $OUT/b32g.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof2560 -o run --output-format csv -- python bench.py --steps 3 --warmup 2 > $OUT/prof2560.log 2>&1
