#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/dbg2
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 env PDDL_TWO_STREAM=0 python scripts/dbg_graph_ov.py > $OUT/ts0.log 2>&1; rc=$?; cat $OUT/ts0.log | tail -30; [ $rc -le 1 ] || exit $rc
timeout -k 10 120 python scripts/dbg_graph_ov.py > $OUT/ts1.log 2>&1; rc=$?; cat $OUT/ts1.log | tail -30; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof2560 -o run --output-format csv -- python bench.py --steps 3 --warmup 2 > $OUT/prof2560.log 2>&1
rc=$?; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/proff32 -o run --output-format csv -- python bench.py --precision fp32 --steps 3 --warmup 2 > $OUT/proff32.log 2>&1
exit $?
