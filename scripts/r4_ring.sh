#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/ring
mkdir -p $OUT
export TMPDIR=/tmp
j() { python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1], d['value'], d['ms_per_step'])" $1; }
for r in 3 5 8; do
  timeout -k 10 200 env PDDL_GRAD_RING=$r python bench.py --batch 32 --steps 60 --warmup 10 > $OUT/b32r$r.json 2> $OUT/b32r$r.err; rc=$?; j $OUT/b32r$r.json; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 200 env PDDL_GRAD_RING=$r python bench.py --batch 32 --steps 60 --warmup 10 --graph 1 > $OUT/b32gr$r.json 2> $OUT/b32gr$r.err; rc=$?; j $OUT/b32gr$r.json; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 200 env PDDL_GRAD_RING=8 python bench.py --batch 256 --steps 20 --warmup 5 --crop 160 > $OUT/b256r8.json 2> $OUT/b256r8.err; rc=$?; j $OUT/b256r8.json
