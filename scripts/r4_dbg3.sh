#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/dbg3
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -v -x --timeout 200 --timeout-method thread -k "c64" > $OUT/eng.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|assert|^E " $OUT/eng.log | head -20; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_runtime.py -v -x --timeout 200 --timeout-method thread > $OUT/rt.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|assert|^E |Fatal" $OUT/rt.log | head -30; exit $rc
