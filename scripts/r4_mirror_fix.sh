#!/bin/bash
# 64-channel 3x3 kernels under HIP-graph capture (the Mirrored entry script's captured first step),
# the GPU suite, smoke, and every entry script at its preset on one GPU.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/mfix
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -v -x --timeout 120 --timeout-method thread -k "c64" > $OUT/kt.log 2>&1
rc=$?; grep -E "FAIL|^E |passed|failed" $OUT/kt.log | head -20; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $OUT/gputests.log 2>&1
rc=$?; tail -3 $OUT/gputests.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?; tail -1 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
bash scripts/strategy_bench.sh 1 30 256
