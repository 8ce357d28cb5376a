#!/bin/bash
# Whole-step A/B over kernel knob sets (PDDL_KNOBS), one bench.py run per set, same box.
#   bash scripts/knob_sweep.sh OUTDIR "bench args" "knobs1" "knobs2" ...   ("-" = defaults)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$1; ARGS=$2; shift 2
mkdir -p $OUT
export TMPDIR=/tmp
j() { python -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]);print(f'{sys.argv[2]:40s} {d[\"value\"]:10.1f} img/s {d[\"ms_per_step\"]:8.3f} ms')" $1 "$2"; }
i=0
for knobs in "$@"; do
  i=$((i+1))
  k=$knobs; [ "$k" = "-" ] && k=""
  PDDL_KNOBS=$k timeout -k 10 300 python bench.py $ARGS > $OUT/run$i.json 2> $OUT/run$i.err || { tail -3 $OUT/run$i.err; exit 1; }
  j $OUT/run$i.json "$knobs"
done
