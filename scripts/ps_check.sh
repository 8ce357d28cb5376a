#!/bin/bash
# PS on one GPU: the GPU PS tests, a 1 PS + 2 worker rehearsal at the reference's batch 32 (roles
# share the card: PDDL_REHEARSE=1), and a HIP API trace of a short rehearsal (host syncs per step).
#   bash scripts/ps_check.sh OUTDIR
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/ps}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_ps.py "tests/test_gpu_runtime.py::test_bench_parameter_server_rehearsal_on_one_gpu" -v -x --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; grep -E "PASS|FAIL|passed|failed" $OUT/tests.log | tail -6; [ $rc -eq 0 ] || exit $rc
for w in bf16 fp32; do
  PDDL_REHEARSE=1 timeout -k 10 300 python bench.py --gpus 3 --strategy ps --ps 1 --batch 32 --steps 200 --ps-wire $w > $OUT/ps_b32_$w.json 2> $OUT/ps_b32_$w.err || { tail -5 $OUT/ps_b32_$w.err; exit 1; }
  python -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]);print(sys.argv[1], d['value'], d.get('ps_service'))" $OUT/ps_b32_$w.json
done
PDDL_REHEARSE=1 timeout -k 10 300 rocprofv3 --hip-trace --output-format csv -d $OUT/trace -o run -- python bench.py --gpus 3 --strategy ps --ps 1 --batch 32 --steps 40 > $OUT/trace.log 2>&1 || { tail -5 $OUT/trace.log; exit 1; }
python scripts/hip_sync_count.py $OUT/trace
