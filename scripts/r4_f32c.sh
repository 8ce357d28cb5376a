#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/f32c
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_f32.py -x -q --timeout 120 --timeout-method thread > $OUT/t.log 2>&1
rc=$?; tail -2 $OUT/t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --precision fp32 --batch 256 --steps 6 --warmup 2 > $OUT/b.json 2> $OUT/b.err || exit $?
cut -c1-200 $OUT/b.json
bash scripts/r4_f32pmc.sh "s4.c0,s3.c2,s2.c2,s4.c2" || exit $?
python scripts/pmc_summary.py gpurun_out/f32pmc > $OUT/pmc_summary.txt 2>&1; cat $OUT/pmc_summary.txt
