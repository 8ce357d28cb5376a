# ad-hoc GPU session (edited per experiment); every step bounded, chained with &&
# current: entry-script sweep (thread-local graph capture) + the graph tests
set -o pipefail
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
true && \
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_runtime.py -k "graph or mirrored" > gpurun_out/ab/graphtests.log 2>&1 && \
bash scripts/strategy_bench.sh 1 30 256 > gpurun_out/ab/strategy.log 2>&1
rc=$?
tail -2 gpurun_out/ab/graphtests.log
cat gpurun_out/strategy_bench.txt
exit $rc
