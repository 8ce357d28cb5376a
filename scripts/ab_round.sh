# ad-hoc GPU session (edited per experiment); every step bounded, chained with &&
# current: register-direct epilogue (igemm_rd) -> kernel numerics, then b1024 / b2048 A/B and a
# kernel-trace profile of the RD build
set -o pipefail
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
b() { local n=$1; shift; timeout -k 10 300 python bench.py "$@" > gpurun_out/ab/$n.log 2>&1; }
true && \
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py > gpurun_out/ab/tests.log 2>&1 && \
b rd1_b1024 --batch 1024 && PDDL_KNOBS=igemm_rd=0 b rd0_b1024 --batch 1024 && \
b rd1_b2048 && PDDL_KNOBS=igemm_rd=0 b rd0_b2048 && b rd1_b1024b --batch 1024 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ab/prof -o run --output-format csv -- python bench.py --batch 1024 --steps 6 --warmup 3 > gpurun_out/ab/prof.log 2>&1
rc=$?
tail -n 3 gpurun_out/ab/tests.log
for f in gpurun_out/ab/*.log; do echo "$f $(grep -h '"value"' $f | cut -c100-160)"; done
exit $rc
