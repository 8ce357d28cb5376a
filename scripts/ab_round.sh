# ad-hoc GPU session (edited per experiment); every step bounded, chained with &&
set -o pipefail
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
b() { local n=$1; shift; timeout -k 10 300 python bench.py "$@" > gpurun_out/ab/$n.log 2>&1; }
p() { local n=$1; shift; timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ab/prof_$n -o run --output-format csv -- python bench.py --steps 4 --warmup 2 "$@" > gpurun_out/ab/prof_$n.log 2>&1; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_fuzz.py tests/test_gpu_engine.py -x -q --timeout 120 > gpurun_out/ab/tests.log 2>&1 && \
b b1024 && b b1024b && p def && b bntrain --bn-mode train --steps 10 --warmup 3
rc=$?
tail -n 3 gpurun_out/ab/tests.log
grep -h '"value"' gpurun_out/ab/*.log | cut -c1-150
exit $rc
