# ad-hoc GPU A/B session (edited per experiment); every step bounded, chained with &&
set -o pipefail
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k maxpool --timeout 120 > gpurun_out/ab/pooltest.log 2>&1 && \
timeout -k 10 300 python bench/pool.py --json gpurun_out/ab/pool.json > gpurun_out/ab/pool.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/ab/bench_default.log 2>&1
rc=$?
cat gpurun_out/ab/pool.log
grep -h '"value"' gpurun_out/ab/bench_*.log | cut -c1-200
exit $rc
