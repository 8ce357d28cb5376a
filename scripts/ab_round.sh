# ad-hoc GPU session (edited per experiment); every step bounded, chained with &&
# current: fp32 (reference precision) and train-BN at larger batches
set -o pipefail
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
b() { local n=$1; shift; timeout -k 10 400 python bench.py "$@" > gpurun_out/ab/$n.log 2>&1; }
true && b fp32_b512 --precision fp32 --batch 512 --steps 8 --warmup 2 && b fp32_b1024 --precision fp32 --batch 1024 --steps 6 --warmup 2 && \
b bnt_b2048 --bn-mode train --batch 2048 --steps 10 --warmup 3
rc=$?
for f in gpurun_out/ab/*.log; do echo "$f $(grep -ho '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"peak_mem_gb": [0-9.]*' $f | tr '\n' ' ') $(grep -m1 Error $f)"; done
exit $rc
