# ad-hoc GPU session (edited per experiment); every step bounded, chained with &&
# current: whole-step HIP graph and batch 2560 against the default, then the PMC counter passes
set -o pipefail
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
b() { local n=$1; shift; timeout -k 10 300 python bench.py "$@" > gpurun_out/ab/$n.log 2>&1; }
true && \
b graph_b1024 --batch 1024 --graph 1 && \
b def_b1024 --batch 1024 && \
bash scripts/pmc_round.sh
rc=$?
for f in gpurun_out/ab/*.log; do echo "$f $(grep -ho '"value": [0-9.]*\|"peak_mem_gb": [0-9.]*' $f | tr '\n' ' ')"; done
exit $rc
