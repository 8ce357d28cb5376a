#!/bin/bash
# PS rehearsal on one GPU (1 PS + 2 workers, b32): worker graphs on / off x gradient-ring depth.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/psring}
mkdir -p $OUT
export TMPDIR=/tmp
for g in 1 0; do for ring in 16 5; do
  PDDL_GRAD_RING=$ring PDDL_REHEARSE=1 timeout -k 10 300 python bench.py --gpus 3 --strategy ps --ps 1 --batch 32 --steps 300 --graph $g > $OUT/g${g}_r${ring}.json 2> $OUT/g${g}_r${ring}.err || { tail -5 $OUT/g${g}_r${ring}.err; exit 1; }
  python -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]);print('graph',sys.argv[2],'ring',sys.argv[3], d['value'])" $OUT/g${g}_r${ring}.json $g $ring
done; done
