#!/bin/bash
# pruned 64-channel 3x3 kernels (8-wave row tiles only): tests + kernel micro-bench + b2560
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/row8b
mkdir -p $OUT
export TMPDIR=/tmp
j() { python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1], d['value'], d['ms_per_step'])" $1; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_engine.py -v -s -x --timeout 200 --timeout-method thread -k "c64 or conv3x3c64" > $OUT/t.log 2>&1
rc=$?; grep -E "FAIL|^E |ratio|c64:" $OUT/t.log | head -20; grep -c PASSED $OUT/t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench/c64.py > $OUT/micro.txt 2>&1 || exit $?
grep -v amdgpu $OUT/micro.txt | grep -v '^{'
timeout -k 10 200 python bench.py --steps 12 --warmup 4 > $OUT/b2560.json 2> $OUT/b2560.err; rc=$?; j $OUT/b2560.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof2560 -o run --output-format csv -- python bench.py --steps 3 --warmup 2 > $OUT/prof2560.log 2>&1
