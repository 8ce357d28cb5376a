#!/bin/bash
# Round 4: b32 two-stream kernel trace + PS bf16-wire rehearsal.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/b32
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --batch 32 --steps 10 --warmup 5 > $OUT/prof.log 2>&1 || exit $?
for w in fp32 bf16 fp32 bf16; do
  timeout -k 10 300 env PDDL_REHEARSE=1 python bench.py --gpus 3 --strategy ps --ps 1 --batch 32 --steps 60 --ps-wire $w > $OUT/ps_$w.out 2> $OUT/ps_$w.err || { echo "ps $w failed"; tail -5 $OUT/ps_$w.err; exit 1; }
  grep '^{' $OUT/ps_$w.out | tail -1 > $OUT/ps_$w.json
  python -c "import json;d=json.load(open('$OUT/ps_$w.json'));print('ps wire $w', d['value'], d.get('ps_service'))" | tee -a $OUT/summary.txt
done
