#!/bin/bash
# Round-4 GPU check: engine parity (ratio prints) then the full GPU suite, each under its own limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -v -s --timeout 200 --timeout-method thread \
  -k "noise_floor or trajectory" > gpurun_out/parity.log 2>&1
rc=$?
grep -E "ratio|passed|failed" gpurun_out/parity.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/gputests.log 2>&1
rc2=$?
tail -15 gpurun_out/gputests.log
exit $rc2
