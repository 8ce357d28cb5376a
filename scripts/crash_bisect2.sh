#!/bin/bash
# crash_bisect.sh, ending in the given test files instead of the Mirrored test (files in order).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$1; shift
mkdir -p $OUT
export TMPDIR=/tmp PDDL_CRASH_TRACE=$PWD/$OUT/crash_trace.txt GLIBC_TUNABLES=glibc.malloc.perturb=165
timeout -k 10 600 python -u -m pytest "$@" -q -m gpu -p no:randomly --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; head -4 $OUT/crash_trace.txt 2>/dev/null; exit $rc
