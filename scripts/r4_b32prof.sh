#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/b32p
mkdir -p $OUT
export TMPDIR=/tmp
j() { python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1], d['value'], d['ms_per_step'])" $1; }
timeout -k 10 200 python bench.py --batch 32 --steps 40 --warmup 10 > $OUT/b32.json 2> $OUT/b32.err; rc=$?; j $OUT/b32.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 env PDDL_TWO_STREAM=0 python bench.py --batch 32 --steps 40 --warmup 10 > $OUT/b32ts0.json 2> $OUT/b32ts0.err; rc=$?; j $OUT/b32ts0.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --batch 32 --steps 10 --warmup 5 > $OUT/prof.log 2>&1
