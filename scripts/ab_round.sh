# ad-hoc GPU session (edited per experiment); every step bounded, chained with &&
# current: final kernel-trace profile of the default bench (b2048) and of b1024
set -o pipefail
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
true && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ab/prof_b2048 -o run --output-format csv -- python bench.py --steps 5 --warmup 3 > gpurun_out/ab/prof_b2048.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ab/prof_b1024 -o run --output-format csv -- python bench.py --batch 1024 --steps 6 --warmup 3 > gpurun_out/ab/prof_b1024.log 2>&1
rc=$?
for f in gpurun_out/ab/*.log; do echo "$f $(grep -ho '"value": [0-9.]*' $f)"; done
exit $rc
