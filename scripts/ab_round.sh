# ad-hoc GPU session (edited per experiment); every step bounded, chained with &&
# current: stride-2 form of the fused conv3 backward (conv2_block3 / conv3_block4) -> kernel
# numerics, engine parity, then b1024 / b2560 A/B against PDDL_FUSE_BWD_S2=0 and a profile
set -o pipefail
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
b() { local n=$1; shift; timeout -k 10 300 python bench.py "$@" > gpurun_out/ab/$n.log 2>&1; }
true && \
timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k bwd1x1 > gpurun_out/ab/t_kernel.log 2>&1 && \
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_engine.py tests/test_gpu_kernels.py > gpurun_out/ab/tests.log 2>&1 && \
b s1 --batch 1024 && PDDL_FUSE_BWD_S2=0 b s0 --batch 1024 && b s1_b2560 && PDDL_FUSE_BWD_S2=0 b s0_b2560 && b s1b --batch 1024 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ab/prof_s1 -o run --output-format csv -- python bench.py --batch 1024 --steps 6 --warmup 3 > gpurun_out/ab/prof_s1.log 2>&1
rc=$?
tail -n 3 gpurun_out/ab/t_kernel.log gpurun_out/ab/tests.log 2>/dev/null
for f in gpurun_out/ab/*.log; do echo "$f $(grep -ho '"value": [0-9.]*\|"peak_mem_gb": [0-9.]*' $f | tr '\n' ' ')"; done
exit $rc
