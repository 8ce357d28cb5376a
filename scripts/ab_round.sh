# ad-hoc GPU session (edited per experiment); every step bounded, chained with &&
set -o pipefail
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
b() { local n=$1; shift; timeout -k 10 300 python bench.py "$@" > gpurun_out/ab/$n.log 2>&1; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_bn_train.py -x -q --timeout 120 > gpurun_out/ab/bntests.log 2>&1 && \
b bntrain --bn-mode train --steps 10 --warmup 3 && \
b b512 --batch 512 --steps 20 --warmup 5 && b b1024 --steps 20 --warmup 5 && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 > gpurun_out/ab/gputests.log 2>&1
rc=$?
tail -n 3 gpurun_out/ab/bntests.log gpurun_out/ab/gputests.log
grep -h '"value"' gpurun_out/ab/*.log | cut -c1-150
grep -ho '"peak_mem_gb": [0-9.]*' gpurun_out/ab/*.log
exit $rc
