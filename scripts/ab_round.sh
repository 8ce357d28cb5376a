# ad-hoc GPU session (edited per experiment); every step bounded, chained with &&
# current: fused projection blocks (conv3 + shortcut as one dual-source GEMM) -> numerics (kernel
# + engine parity suites), then b1024 / b2048 A/B against PDDL_FUSE_PROJ=0 and a profile
set -o pipefail
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
b() { local n=$1; shift; timeout -k 10 300 python bench.py "$@" > gpurun_out/ab/$n.log 2>&1; }
true && \
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_engine.py tests/test_gpu_kernels.py > gpurun_out/ab/tests.log 2>&1 && \
b f1 --batch 1024 && PDDL_FUSE_PROJ=0 b f0 --batch 1024 && b f1_b2048 && PDDL_FUSE_PROJ=0 b f0_b2048 && b f1b_b2048 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ab/prof_f1 -o run --output-format csv -- python bench.py --batch 1024 --steps 6 --warmup 3 > gpurun_out/ab/prof_f1.log 2>&1
rc=$?
tail -n 3 gpurun_out/ab/tests.log
for f in gpurun_out/ab/*.log; do echo "$f $(grep -ho '"value": [0-9.]*\|"peak_mem_gb": [0-9.]*' $f | tr '\n' ' ')"; done
exit $rc
