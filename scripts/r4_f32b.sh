#!/bin/bash
# fp32 conv kernels after the tile-width template + asm fragment reads: tests, micro-bench, step
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/f32b
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_f32.py -v -x --timeout 120 --timeout-method thread > $OUT/t.log 2>&1
rc=$?; grep -E "PASS|FAIL|^E " $OUT/t.log | head -30; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench/f32.py > $OUT/micro.txt 2>&1 || exit $?
tail -4 $OUT/micro.txt
timeout -k 10 200 python bench.py --precision fp32 --batch 256 --steps 6 --warmup 2 > $OUT/b.json 2> $OUT/b.err || exit $?
cut -c1-200 $OUT/b.json
