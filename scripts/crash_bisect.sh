#!/bin/bash
# One pytest process over the given test files, then the Mirrored graphed-step test in the same
# process (the long-lived-process condition of the hipGraphLaunch crash); glibc frees are
# perturbed so a use-after-free reads a recognisable pattern.   crash_bisect.sh OUT files...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$1; shift
mkdir -p $OUT
export TMPDIR=/tmp PDDL_CRASH_TRACE=$PWD/$OUT/crash_trace.txt GLIBC_TUNABLES=glibc.malloc.perturb=165
timeout -k 10 600 python -u -m pytest "$@" "tests/test_gpu_runtime.py::test_mirrored_graphed_step_matches_eager" \
  -q -m gpu --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; head -8 $OUT/crash_trace.txt 2>/dev/null; exit $rc
