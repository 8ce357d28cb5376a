# ad-hoc GPU session (edited per experiment); every step bounded, chained with &&
# current: unrolled 3x3 halo tap masks -> kernel numerics, b1024 bench x2 + kernel-trace profile
set -o pipefail
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
b() { local n=$1; shift; timeout -k 10 300 python bench.py "$@" > gpurun_out/ab/$n.log 2>&1; }
prof() { local n=$1; shift; timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ab/prof_$n -o run --output-format csv -- python bench.py --batch 1024 --steps 6 --warmup 3 > gpurun_out/ab/prof_$n.log 2>&1; }
true && \
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_engine.py > gpurun_out/ab/tests.log 2>&1 && \
b h1 --batch 1024 && b h1b --batch 1024 && b h1_b2048 && prof h1
rc=$?
tail -n 2 gpurun_out/ab/tests.log
for f in gpurun_out/ab/*.log; do echo "$f $(grep -ho '"value": [0-9.]*' $f)"; done
exit $rc
