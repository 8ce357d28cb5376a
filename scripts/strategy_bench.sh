#!/bin/bash
# Throughput of every reference entry point on one node through the real
# CLI / Trainer / strategy stack, synthetic data, the presets' own crop sizes, no checkpoint
# write.  Prints one "strategy gpus img/s" line per run into gpurun_out/strategy_bench.txt.
#
#   bash scripts/strategy_bench.sh [NGPU=1] [STEPS=30] [BATCH=256]
#
# NGPU > 1 is meant for an 8-GPU node (Mirrored uses every visible GPU in one process; Horovod
# and MultiWorkerMirrored run one rank per GPU under torchrun; the PS job runs 2 PS + NGPU-2
# workers).  On one GPU every role shares the card (PS: 1 PS + 1 worker).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
NGPU=${1:-1}; STEPS=${2:-30}; BATCH=${3:-256}
mkdir -p gpurun_out
OUT=gpurun_out/strategy_bench.txt
COMMON="--data synthetic --epochs 1 --steps-per-epoch $STEPS --validation-steps 0 --batch-size $BATCH --no-save"
TR="python -m torch.distributed.run --nnodes=1 --nproc-per-node $NGPU --master-addr 127.0.0.1 --master-port 29611"
run() {  # name gpus timeout cmd...
  local name=$1 g=$2 t=$3; shift 3
  echo "=== $name ($g GPU)"
  timeout -k 10 "$t" "$@" > "gpurun_out/sb_$name.log" 2>&1
  local rc=$?
  local ips
  ips=$(grep -o "[0-9.]* img/s" "gpurun_out/sb_$name.log" | tail -1)
  echo "$name $g ${ips:-none} rc=$rc" | tee -a "$OUT"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
: > "$OUT"
run single 1 300 python -u imagenet-resnet50.py $COMMON
run mirrored "$NGPU" 300 python -u imagenet-resnet50-mirror.py $COMMON
run horovod "$NGPU" 300 $TR imagenet-resnet50-hvd.py $COMMON
run multiworker "$NGPU" 300 $TR imagenet-resnet50-multiworkers.py $COMMON
if [ "$NGPU" -ge 3 ]; then NPS=2; else NPS=1; fi
NW=$(( NGPU > NPS ? NGPU - NPS : 1 ))
run ps "$NGPU" 400 python -u imagenet-resnet50-ps.py --ps $NPS --worker $NW $COMMON
cat "$OUT"
