#!/bin/bash
# Interleaved A/B of kernel-knob settings on the headline step (one process per run, alternating
# arms R rounds):   bash scripts/ab_knobs.sh OUTDIR ROUNDS "knobsA" "knobsB" [bench args...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$1; R=$2; A=$3; B=$4; shift 4
mkdir -p $OUT
for r in $(seq 1 $R); do
  for arm in A B; do
    k=$A; [ $arm = B ] && k=$B
    PDDL_KNOBS="$k" timeout -k 10 240 python bench.py --steps 10 --warmup 3 "$@" > $OUT/${arm}_$r.json 2> $OUT/${arm}_$r.err || exit $?
    python -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]);print(sys.argv[2], sys.argv[3], d['value'], d['ms_per_step'])" $OUT/${arm}_$r.json $arm "$k"
  done
done
