#!/bin/bash
# PMC passes (bench/pmc.txt groups, one rocprofv3 run each) over a micro-benchmark:
#   bash scripts/pmc_bench.sh OUTDIR python bench/stem.py --iters 3
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$1; shift
mkdir -p $OUT
export TMPDIR=/tmp
i=0
while read -r tag counters; do
  [ "$tag" = "pmc:" ] || continue
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --pmc $counters --output-format csv -d $OUT/pmc_$i -o run -- "$@" > $OUT/pmc_$i.log 2>&1 || exit $?
done < bench/pmc.txt
python scripts/pmc_summary.py $OUT
