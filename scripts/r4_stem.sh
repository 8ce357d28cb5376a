#!/bin/bash
# Round 4: fused stem (conv1 + max-pool) kernel test, engine tests, bench + per-layer trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/stem
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread -k "stem_pool" > $OUT/kt.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|assert" $OUT/kt.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py -x -q --timeout 200 --timeout-method thread > $OUT/eng.log 2>&1
rc=$?; tail -3 $OUT/eng.log
[ $rc -eq 0 ] || exit $rc
for v in 1 0 1; do
  timeout -k 10 240 env PDDL_FUSE_STEM=$v python bench.py --steps 12 --warmup 4 > $OUT/b$v.json 2>$OUT/b$v.err || exit $?
  python -c "import json;d=json.load(open('$OUT/b$v.json'));print('fuse_stem=$v', d['value'], d['ms_per_step'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --steps 3 --warmup 2 > $OUT/prof.log 2>&1
