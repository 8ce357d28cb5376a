# ad-hoc GPU session (edited per experiment); every step bounded, chained with &&
# current: per-GPU batch 2560 (fits 2^31 elements now that conv2_block1's c1+shortcut split
# output is gone) vs the 2048 default, back to back
set -o pipefail
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
b() { local n=$1; shift; timeout -k 10 300 python bench.py "$@" > gpurun_out/ab/$n.log 2>&1; }
b b2048 && b b2560 --batch 2560 && b b2048b && b b2560b --batch 2560
rc=$?
for f in gpurun_out/ab/*.log; do echo "$f $(grep -ho '"value": [0-9.]*\|"peak_mem_gb": [0-9.]*\|"ms_per_step": [0-9.]*' $f | tr '\n' ' ')"; done
tail -3 gpurun_out/ab/b2560.log
exit $rc
