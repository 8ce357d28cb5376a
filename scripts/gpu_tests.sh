#!/bin/bash
# GPU tests: optional focused file(s) first, then the whole GPU suite in one process.
#   bash scripts/gpu_tests.sh OUTDIR [test files...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/tests}; shift
mkdir -p $OUT
export TMPDIR=/tmp
export PDDL_CRASH_TRACE=$PWD/$OUT/crash_trace.txt
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u -m pytest "$@" -v -x --timeout 200 --timeout-method thread > $OUT/focused.log 2>&1
  rc=$?; grep -E "PASS|FAIL|^E |passed|failed|crash trace" $OUT/focused.log | tail -30; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rf --timeout 200 --timeout-method thread > $OUT/gputests.log 2>&1
rc=$?; tail -4 $OUT/gputests.log; exit $rc
