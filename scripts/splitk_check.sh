#!/bin/bash
# Split-K in-kernel reduction: kernel tests, then b32 / b32-crop160 graphed steps with the fused
# reduction on and off (igemm_sk_fused knob via PDDL_KNOBS), then the whole GPU suite.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/splitk}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -k "splitk" -v -x --timeout 200 --timeout-method thread > $OUT/kt.log 2>&1
rc=$?; grep -E "passed|failed|FAIL" $OUT/kt.log | tail -4; [ $rc -eq 0 ] || exit $rc
j() { python -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]);print(sys.argv[1], d['value'], d['ms_per_step'])" $1; }
for f in 1 0; do
  for c in 224 160; do
    PDDL_KNOBS=igemm_sk_fused=$f timeout -k 10 240 python bench.py --batch 32 --crop $c --steps 60 --warmup 10 --graph 1 > $OUT/b32c${c}_f$f.json 2> $OUT/b32c${c}_f$f.err || { tail -3 $OUT/b32c${c}_f$f.err; exit 1; }
    j $OUT/b32c${c}_f$f.json
  done
done
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $OUT/gputests.log 2>&1
rc=$?; tail -2 $OUT/gputests.log; exit $rc
