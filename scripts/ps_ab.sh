#!/bin/bash
# PS rehearsal A/B on one GPU (1 PS + 2 workers, b32): graphs on / off x ticket block 16 / 1.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/psab}
mkdir -p $OUT
export TMPDIR=/tmp
for g in 1 0; do for blk in 16 1; do
  PDDL_PS_TICKET_BLOCK=$blk PDDL_REHEARSE=1 timeout -k 10 300 python bench.py --gpus 3 --strategy ps --ps 1 --batch 32 --steps 300 --graph $g > $OUT/g${g}_b${blk}.json 2> $OUT/g${g}_b${blk}.err || { tail -5 $OUT/g${g}_b${blk}.err; exit 1; }
  python -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]);print('graph',sys.argv[2],'block',sys.argv[3], d['value'], {k: round(v,3) for k,v in d['ps_service'][0].items()})" $OUT/g${g}_b${blk}.json $g $blk
done; done
