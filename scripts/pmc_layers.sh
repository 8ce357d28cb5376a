#!/bin/bash
# Per-layer HBM traffic of a training step: one rocprofv3 counter pass per byte counter
# (WRITE_SIZE; FETCH_SIZE) over a short bench run, for the given knob settings.
#   bash scripts/pmc_layers.sh TAG "knobs"
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=$1; knobs=$2
mkdir -p gpurun_out/pmcl
for P in WRITE_SIZE FETCH_SIZE; do
  PDDL_KNOBS="$knobs" timeout -s KILL 120 rocprofv3 --pmc $P -d gpurun_out/pmcl/${tag}_$P -o run --output-format csv -- \
    python bench.py --batch 1024 --steps 2 --warmup 1 > gpurun_out/pmcl/${tag}_$P.log 2>&1 || exit 1
done
