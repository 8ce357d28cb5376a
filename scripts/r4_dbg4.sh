#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/dbg4
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -v -s --timeout 200 --timeout-method thread -k "c64" > $OUT/eng.log 2>&1
rc=$?; grep -E "PASS|FAIL|c64 variant" $OUT/eng.log | head -20; [ $rc -le 1 ] || exit $rc
for v in 0 1 2; do
  if [ $v = 0 ]; then envs="PDDL_C64=0"; else envs="PDDL_C64_MIN_M=1 PDDL_KNOBS=c64=$v"; fi
  echo "== $envs" >> $OUT/parity.log
  timeout -k 10 300 env $envs python -u -m pytest tests/test_gpu_engine.py -v -s --timeout 200 --timeout-method thread -k "noise_floor" >> $OUT/parity.log 2>&1
  rc=$?; [ $rc -le 1 ] || exit $rc
done
grep -E "^==|ratio|passed|failed" $OUT/parity.log
