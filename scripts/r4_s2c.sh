#!/bin/bash
# compact stride-2-grid outputs of the blocks feeding a downsampling block: tests, A/B bench, trace
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/s2c
mkdir -p $OUT
export TMPDIR=/tmp
j() { python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1], d['value'], d['ms_per_step'])" $1; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -v -x --timeout 120 --timeout-method thread -k "up2 or stride2_residual" > $OUT/kt.log 2>&1
rc=$?; grep -E "PASS|FAIL|^E " $OUT/kt.log | head -20; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -v -s --timeout 200 --timeout-method thread -k "s2_fed or graphed_step or two_stream" > $OUT/eng.log 2>&1
rc=$?; grep -E "PASS|FAIL|^E |s2c:|ratio" $OUT/eng.log | head -20; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --steps 12 --warmup 4 > $OUT/b2560.json 2> $OUT/b2560.err; rc=$?; j $OUT/b2560.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 env PDDL_S2C=0 python bench.py --steps 12 --warmup 4 > $OUT/b2560off.json 2> $OUT/b2560off.err; rc=$?; j $OUT/b2560off.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --steps 12 --warmup 4 > $OUT/b2560b.json 2> $OUT/b2560b.err; rc=$?; j $OUT/b2560b.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --batch 32 --steps 60 --warmup 10 --graph 1 > $OUT/b32g.json 2> $OUT/b32g.err; rc=$?; j $OUT/b32g.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof2560 -o run --output-format csv -- python bench.py --steps 3 --warmup 2 > $OUT/prof2560.log 2>&1
