#!/bin/bash
# b2560 A/B of igemm tile-selection knobs (PDDL_KNOBS), interleaved, same box
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/knobs
mkdir -p $OUT
j() { python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1], d['value'], d['ms_per_step'])" $1; }
run() { local tag=$1; local k=$2; timeout -k 10 200 env PDDL_KNOBS="$k" python bench.py --steps 12 --warmup 4 > $OUT/$tag.json 2> $OUT/$tag.err || { tail -3 $OUT/$tag.err; return 1; }; j $OUT/$tag.json; }
for r in 1 2; do
  run base$r "" && run m256_$r "igemm8_min_n=256" && run ns2_$r "igemm_ns1_kt=8" || exit 1
done
