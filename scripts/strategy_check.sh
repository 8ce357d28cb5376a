#!/bin/bash
# Strategy-level GPU checks on one GPU: the entry-script sweep at b256 (crop presets), Mirrored
# and single at the reference's batch 32, the Horovod preset (b32, crop 160) through the Trainer
# eager / whole-step graph.
#   bash scripts/strategy_check.sh OUTDIR
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/strategy}
mkdir -p $OUT
export TMPDIR=/tmp
bash scripts/strategy_bench.sh 1 30 256 || exit $?
cp gpurun_out/strategy_bench.txt $OUT/
j() { python -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]);print(sys.argv[1], d['value'], d['ms_per_step'])" $1; }
b() { local tag=$1; shift; timeout -k 10 240 python bench.py "$@" > $OUT/$tag.json 2> $OUT/$tag.err || { echo "$tag failed"; tail -3 $OUT/$tag.err; return 1; }; j $OUT/$tag.json; }
b mirrored_b32 --strategy mirrored --batch 32 --steps 60 --warmup 10 && \
b mirrored_b32c244 --strategy mirrored --batch 32 --crop 244 --steps 60 --warmup 10 && \
b single_b32g --batch 32 --steps 60 --warmup 10 --graph 1 || exit 1
H="--data synthetic --epochs 1 --steps-per-epoch 80 --validation-steps 0 --batch-size 32 --no-save"
for mode in eager whole; do
  case $mode in
    eager) env= ; extra= ;;
    whole) env= ; extra="--graphs" ;;
  esac
  timeout -k 10 300 env $env python -u imagenet-resnet50-hvd.py $H $extra > $OUT/hvd_$mode.log 2>&1
  rc=$?; echo "hvd b32 crop160 $mode: $(grep -o '[0-9.]* img/s' $OUT/hvd_$mode.log | tail -1) rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
