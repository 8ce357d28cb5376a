# ad-hoc GPU session (edited per experiment); every step bounded, chained with &&
# current: descriptor rebasing -> kernel numerics (incl. > 2 GiB operands), then b1024 / b1536 / b2048
set -o pipefail
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
b() { local n=$1; shift; timeout -k 10 300 python bench.py "$@" > gpurun_out/ab/$n.log 2>&1; }
true && \
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_f32.py > gpurun_out/ab/tests.log 2>&1 && \
b b1024 --batch 1024 && b b1536 --batch 1536 && b b2048 --batch 2048 && b b1024b --batch 1024 && b b2048b --batch 2048
rc=$?
tail -n 3 gpurun_out/ab/tests.log
for f in gpurun_out/ab/b*.log; do echo "$f $(grep -h '"value"' $f | cut -c100-160)"; done
exit $rc
