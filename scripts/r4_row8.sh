#!/bin/bash
# 8-wave 64-channel 3x3 row kernel (c64 = 3): tests, kernel A/B, b2560 A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/row8
mkdir -p $OUT
export TMPDIR=/tmp
j() { python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1], d['value'], d['ms_per_step'])" $1; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -v -x --timeout 120 --timeout-method thread -k "conv3x3c64_ring" > $OUT/kt.log 2>&1
rc=$?; grep -E "FAIL|^E " $OUT/kt.log | head -20; grep -c PASSED $OUT/kt.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -v -s -x --timeout 200 --timeout-method thread -k "c64" > $OUT/eng.log 2>&1
rc=$?; grep -E "PASS|FAIL|^E |ratio" $OUT/eng.log | head -20; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench/c64.py > $OUT/micro.txt 2>&1 || exit $?
grep -v amdgpu $OUT/micro.txt | grep -v '^{'
for r in 1 2; do
  timeout -k 10 200 env PDDL_KNOBS="c64=3" python bench.py --steps 12 --warmup 4 > $OUT/r8_$r.json 2> $OUT/r8_$r.err; rc=$?; j $OUT/r8_$r.json; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 200 python bench.py --steps 12 --warmup 4 > $OUT/base_$r.json 2> $OUT/base_$r.err; rc=$?; j $OUT/base_$r.json; [ $rc -eq 0 ] || exit $rc
done
