#!/bin/bash
# Round 4: two-stream with gradient rings + optimizer overlapped with backward: tests + benches.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/ov
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 python scripts/dbg_c64w.py > $OUT/dbg.log 2>&1; rc=$?; [ $rc -le 1 ] || exit $rc
timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread -k "c64 or stem_pool" > $OUT/kt.log 2>&1
rc=$?; grep -E "FAIL|Error|passed|failed|assert" $OUT/kt.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_f32.py -x -v --timeout 120 --timeout-method thread > $OUT/f32.log 2>&1
rc=$?; grep -E "FAIL|Error|passed|failed|assert" $OUT/f32.log | tail -8
[ $rc -eq 0 ] || exit $rc
for cfg in "PDDL_OVERLAP_OPT=0" "PDDL_TWO_STREAM=0" "PDDL_FUSE_STEM=0" "X=1"; do
  echo "== $cfg" >> $OUT/graphdbg.log
  timeout -k 10 120 env $cfg python -u -m pytest tests/test_gpu_engine.py -q --timeout 100 --timeout-method thread -k "graphed_step or two_stream or overlapped" >> $OUT/graphdbg.log 2>&1
  rc=$?; [ $rc -le 1 ] || exit $rc
done
grep -E "^==|passed|failed" $OUT/graphdbg.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py -v --timeout 200 --timeout-method thread > $OUT/eng.log 2>&1
rc=$?; grep -E "FAIL|Error|passed|failed" $OUT/eng.log | tail -5
[ $rc -le 1 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_runtime.py tests/test_gpu_multirank.py -x -q --timeout 300 --timeout-method thread > $OUT/rt.log 2>&1
rc=$?; tail -3 $OUT/rt.log
[ $rc -le 1 ] || exit $rc
run() {  # tag env... -- args...
  local tag=$1; shift; local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  timeout -k 10 240 env "${envs[@]}" python bench.py "$@" > $OUT/$tag.json 2> $OUT/$tag.err || { echo "$tag rc=$?"; tail -3 $OUT/$tag.err; return 1; }
  python -c "import json;d=json.load(open('$OUT/$tag.json'));print('$tag', d['value'], d['ms_per_step'])" | tee -a $OUT/summary.txt
}
run b2560 X=1 -- --steps 12 --warmup 4 && \
run b2560_c64off PDDL_C64=0 -- --steps 12 --warmup 4 && \
run b2560_c64w PDDL_C64W=1 -- --steps 12 --warmup 4 && \
run f32_v1 X=1 -- --precision fp32 --steps 10 --warmup 3 && \
run f32_v0 PDDL_KNOBS=conv_f32=0 -- --precision fp32 --steps 10 --warmup 3 && \
run b32_ov1 X=1 -- --batch 32 --steps 40 --warmup 10 && \
run b32_ov0 PDDL_OVERLAP_OPT=0 -- --batch 32 --steps 40 --warmup 10 && \
run b32g_ov1 X=1 -- --batch 32 --steps 40 --warmup 10 --graph 1 && \
run b32c160 X=1 -- --batch 32 --crop 160 --steps 40 --warmup 10 && \
run b32c160g X=1 -- --batch 32 --crop 160 --steps 40 --warmup 10 --graph 1 && \
run b256c160 X=1 -- --batch 256 --crop 160 --steps 20 --warmup 5 && \
run b1024 X=1 -- --batch 1024 --steps 12 --warmup 4
rc=$?
exit $rc
