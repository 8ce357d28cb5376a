#!/bin/bash
# PS rehearsal (1 PS + 2 workers on one GPU, b32): wire dtype x worker graphs, same box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/psdef}
mkdir -p $OUT
export TMPDIR=/tmp
for w in fp32 bf16; do for g in 0 1; do
  PDDL_REHEARSE=1 timeout -k 10 300 python bench.py --gpus 3 --strategy ps --ps 1 --batch 32 --steps 300 --graph $g --ps-wire $w > $OUT/${w}_g$g.json 2> $OUT/${w}_g$g.err || { tail -5 $OUT/${w}_g$g.err; exit 1; }
  python -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]);print('wire',sys.argv[2],'graph',sys.argv[3], d['value'])" $OUT/${w}_g$g.json $w $g
done; done
