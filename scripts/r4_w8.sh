#!/bin/bash
# 8-wave 64-channel 3x3 weight gradient: tests, kernel A/B, b2560 A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/w8
mkdir -p $OUT
export TMPDIR=/tmp
j() { python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1], d['value'], d['ms_per_step'])" $1; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_engine.py -v -s -x --timeout 200 --timeout-method thread -k "c64 or conv3x3c64" > $OUT/t.log 2>&1
rc=$?; grep -E "FAIL|^E |ratio|c64:" $OUT/t.log | head -20; grep -c PASSED $OUT/t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench/c64.py > $OUT/micro.txt 2>&1 || exit $?
grep -v amdgpu $OUT/micro.txt | grep -v '^{'
for r in 1 2; do
  timeout -k 10 200 python bench.py --steps 12 --warmup 4 > $OUT/w8_$r.json 2> $OUT/w8_$r.err; rc=$?; j $OUT/w8_$r.json; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 200 env PDDL_KNOBS="c64w8=0" python bench.py --steps 12 --warmup 4 > $OUT/w4_$r.json 2> $OUT/w4_$r.err; rc=$?; j $OUT/w4_$r.json; [ $rc -eq 0 ] || exit $rc
done
