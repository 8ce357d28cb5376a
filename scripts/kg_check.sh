#!/bin/bash
# In-workgroup split-K (igemm k-groups): kernel tests, then b32 graphed step times (crop 224 / 160)
# over the k-group knobs, then a kernel trace of the default plan.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/kg}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -k "splitk" -v -x --timeout 200 --timeout-method thread > $OUT/kt.log 2>&1
rc=$?; grep -E "passed|failed|FAIL|Error" $OUT/kt.log | tail -6; [ $rc -eq 0 ] || exit $rc
j() { python -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]);print(sys.argv[1], d['value'], d['ms_per_step'])" $1; }
for knobs in "igemm_kg=0,igemm_sk_rw=1" "igemm_kg=0" "igemm_kg=1" "igemm_kg=4,igemm_kg_ks=1" "igemm_kg=3,igemm_kg_ks=1" "igemm_kg=2,igemm_kg_ks=1" "igemm_kg=4,igemm_kg_ks=2"; do
  for c in 224 160; do
    f=$OUT/b32c${c}_$(echo $knobs | tr ',=' '__').json
    PDDL_KNOBS=$knobs timeout -k 10 240 python bench.py --batch 32 --crop $c --steps 60 --warmup 10 --graph 1 > $f 2> $f.err || { tail -3 $f.err; exit 1; }
    j $f
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run -- python bench.py --batch 32 --steps 30 --warmup 10 --graph 0 > $OUT/trace.log 2>&1 || exit $?
t=$(find $OUT/trace -name "run_kernel_trace.csv" | head -1)
python scripts/step_span.py $t adam_kernel 25
