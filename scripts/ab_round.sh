# ad-hoc GPU session: max-pool forward with two windows in flight per wave -> pool numerics,
# then a b1024 kernel trace (maxpool_fwd was 532-534 us in every round-3 profile)
set -o pipefail
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "pool" > gpurun_out/ab/t_pool.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ab/prof_p -o run --output-format csv -- python bench.py --batch 1024 --steps 6 --warmup 3 > gpurun_out/ab/prof_p.log 2>&1
rc=$?
tail -2 gpurun_out/ab/t_pool.log
grep -h '"value"' gpurun_out/ab/prof_p.log | grep -o '"value": [0-9.]*'
exit $rc
