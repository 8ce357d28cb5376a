# ad-hoc GPU session (edited per experiment); every step bounded, chained with &&
# current: fused stage-2 conv3 backward (bwd1x1.hip) -> kernel numerics, engine parity, then
# b1024 / b2048 A/B against PDDL_FUSE_BWD=0 and a profile
set -o pipefail
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
b() { local n=$1; shift; timeout -k 10 300 python bench.py "$@" > gpurun_out/ab/$n.log 2>&1; }
true && \
timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k bwd1x1 > gpurun_out/ab/t_kernel.log 2>&1 && \
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_engine.py tests/test_gpu_kernels.py > gpurun_out/ab/tests.log 2>&1 && \
b w1 --batch 1024 && PDDL_FUSE_BWD=2 b w2 --batch 1024 && b w1_b2048 && PDDL_FUSE_BWD=2 b w2_b2048 && b w1b --batch 1024 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ab/prof_w1 -o run --output-format csv -- python bench.py --batch 1024 --steps 6 --warmup 3 > gpurun_out/ab/prof_w1.log 2>&1
rc=$?
tail -n 3 gpurun_out/ab/t_kernel.log gpurun_out/ab/tests.log 2>/dev/null
for f in gpurun_out/ab/*.log; do echo "$f $(grep -ho '"value": [0-9.]*\|"peak_mem_gb": [0-9.]*' $f | tr '\n' ' ')"; done
exit $rc
