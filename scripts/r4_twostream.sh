#!/bin/bash
# Round 4: two-stream backward (weight gradients on a side stream) -- tests + small-batch benches.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/ts
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py -x -v --timeout 200 --timeout-method thread > $OUT/eng.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|passed|failed" $OUT/eng.log | tail -20
[ $rc -eq 0 ] || exit $rc
run() {  # tag env... -- args...
  local tag=$1; shift; local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  timeout -k 10 240 env "${envs[@]}" python bench.py "$@" > $OUT/$tag.json 2> $OUT/$tag.err || { echo "$tag rc=$?"; tail -3 $OUT/$tag.err; return 1; }
  python -c "import json;d=json.load(open('$OUT/$tag.json'));print('$tag', d['value'], d['ms_per_step'])" | tee -a $OUT/summary.txt
}
run b32_ts1 PDDL_TWO_STREAM=1 -- --batch 32 --steps 40 --warmup 10 && \
run b32_ts0 PDDL_TWO_STREAM=0 -- --batch 32 --steps 40 --warmup 10 && \
run b32g_ts1 PDDL_TWO_STREAM=1 -- --batch 32 --steps 40 --warmup 10 --graph 1 && \
run b32g_ts0 PDDL_TWO_STREAM=0 -- --batch 32 --steps 40 --warmup 10 --graph 1 && \
run b32c160_ts1 PDDL_TWO_STREAM=1 -- --batch 32 --crop 160 --steps 40 --warmup 10 && \
run b32c160_ts0 PDDL_TWO_STREAM=0 -- --batch 32 --crop 160 --steps 40 --warmup 10 && \
run b256c160_ts1 PDDL_TWO_STREAM=1 -- --batch 256 --crop 160 --steps 20 --warmup 5 && \
run b256c160_ts0 PDDL_TWO_STREAM=0 -- --batch 256 --crop 160 --steps 20 --warmup 5 && \
run b256_ts1 PDDL_TWO_STREAM=1 -- --batch 256 --steps 20 --warmup 5 && \
run b256_ts0 PDDL_TWO_STREAM=0 -- --batch 256 --steps 20 --warmup 5 && \
run b1024_ts1 PDDL_TWO_STREAM=1 -- --batch 1024 --steps 12 --warmup 4 && \
run b1024_ts0 PDDL_TWO_STREAM=0 -- --batch 1024 --steps 12 --warmup 4 && \
run b2560_ts1 PDDL_TWO_STREAM=1 -- --steps 12 --warmup 4 && \
run b2560_ts0 PDDL_TWO_STREAM=0 -- --steps 12 --warmup 4
# PS bf16 wire: unit tests, then the 1 PS + 2 worker rehearsal at b32 with both wires
timeout -k 10 200 python -u -m pytest tests/test_gpu_ps.py -x -v --timeout 120 --timeout-method thread > $OUT/ps.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error" $OUT/ps.log | head
[ $rc -eq 0 ] || exit $rc
for w in fp32 bf16 fp32 bf16; do
  timeout -k 10 300 env PDDL_REHEARSE=1 python bench.py --gpus 3 --strategy ps --ps 1 --batch 32 --steps 60 --ps-wire $w > $OUT/ps_$w.json 2> $OUT/ps_$w.err || { echo "ps $w failed"; tail -5 $OUT/ps_$w.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/ps_$w.json'));print('ps wire $w', d['value'], d.get('ps_service'))" | tee -a $OUT/summary.txt
done
