#!/bin/bash
# 64-channel 3x3 kernels: tests + kernel micro-bench + b2560 A/B against the previous build's numbers
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/c64b
mkdir -p $OUT
export TMPDIR=/tmp
j() { python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1], d['value'], d['ms_per_step'])" $1; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_engine.py -v -x --timeout 120 --timeout-method thread -k "c64 or conv3x3c64" > $OUT/kt.log 2>&1
rc=$?; grep -E "PASS|FAIL|^E " $OUT/kt.log | head -30; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench/c64.py > $OUT/micro.txt 2>&1 || exit $?
cat $OUT/micro.txt | grep -v amdgpu
timeout -k 10 200 python bench.py --steps 12 --warmup 4 > $OUT/b2560.json 2> $OUT/b2560.err; rc=$?; j $OUT/b2560.json; [ $rc -eq 0 ] || exit $rc
