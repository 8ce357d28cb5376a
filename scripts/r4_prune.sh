#!/bin/bash
# after pruning rejected variants (stem-pool first form, dual-source c3c1, 4-wave c64 wgrad): the
# affected kernel and engine tests, the stem fused-vs-unfused check, b2560
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/prune
mkdir -p $OUT
export TMPDIR=/tmp
j() { python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1], d['value'], d['ms_per_step'])" $1; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_engine.py -v -s -x --timeout 200 --timeout-method thread -k "c3c1 or stem or c64 or conv3x3c64 or graphed or two_stream or noise_floor" > $OUT/t.log 2>&1
rc=$?; grep -E "FAIL|^E |ratio|c3c1:|c64:" $OUT/t.log | head -20; grep -c PASSED $OUT/t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u bench/stem.py > $OUT/stem.txt 2>&1 || exit $?
grep -v amdgpu $OUT/stem.txt
timeout -k 10 200 python bench.py --steps 12 --warmup 4 > $OUT/b2560.json 2> $OUT/b2560.err; rc=$?; j $OUT/b2560.json; [ $rc -eq 0 ] || exit $rc
