# ad-hoc GPU A/B session (edited per experiment); every step bounded, chained with &&
set -o pipefail
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
SO=parallel-and-distributed-deep-learning_amd/_pddl_native.cpython-310-x86_64-linux-gnu.so
prof() {  # name knobs
  PDDL_KNOBS=$2 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/ab/prof_$1 -o run --output-format csv -- python bench.py --steps 4 --warmup 2 > gpurun_out/ab/prof_$1.log 2>&1
}
bench() { PDDL_KNOBS=$2 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/ab/bench_$1.log 2>&1; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "wgrad" --timeout 120 > gpurun_out/ab/wgtest.log 2>&1 && \
bench def "" && prof def "" && cp ab_so/minb4.so $SO && bench minb4 "" && prof minb4 "" && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_fuzz.py -x -q --timeout 120 > gpurun_out/ab/minb4_tests.log 2>&1
rc=$?
tail -n 2 gpurun_out/ab/wgtest.log gpurun_out/ab/minb4_tests.log
grep -h '"value"' gpurun_out/ab/bench_*.log | cut -c1-200
exit $rc
