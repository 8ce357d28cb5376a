#!/bin/bash
# One layer at two batch sizes: time per launch and counters (is the small batch slower per
# image, and why).  bash scripts/scale_probe.sh OUTDIR
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/scale}
mkdir -p $OUT
export TMPDIR=/tmp
for s in 256,14,256,256,3,1,1 2560,14,256,256,3,1,1 1024,14,256,256,3,1,1; do
  timeout -k 10 120 python scripts/kprobe.py --op fwd --shape $s --iters 20 || exit 1
done
P1="SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_MFMA"
P2="TCC_HIT_sum TCC_MISS_sum"
for s in 256,14,256,256,3,1,1 2560,14,256,256,3,1,1; do
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $P -d $OUT/pmc_${s//,/_}_$i -o run --output-format csv -- \
      python scripts/kprobe.py --op fwd --shape $s --iters 5 > $OUT/log_${s//,/_}_$i.log 2>&1 || exit 1
  done
done
python - "$OUT" <<'PY'
import csv, glob, sys, collections
root = sys.argv[1]
for d in sorted(glob.glob(root + "/pmc_*")):
    agg = collections.defaultdict(list)
    for f in glob.glob(d + "/**/run_counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "igemm" in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(d.split("/")[-1], {k: round(sum(v) / len(v), 1) for k, v in agg.items()})
PY
