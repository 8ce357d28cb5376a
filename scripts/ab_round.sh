# ad-hoc GPU A/B session (edited per experiment); every step bounded, chained with &&
set -o pipefail
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_fuzz.py -x -q -k n64 --timeout 120 > gpurun_out/ab/n64test.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_engine.py -x -q --timeout 120 > gpurun_out/ab/kerneltests.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/ab/bench_default.log 2>&1 && \
PDDL_KNOBS=igemm_n64=3 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/ab/bench_n64_3.log 2>&1 && \
PDDL_KNOBS=igemm_n64=6 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/ab/bench_n64_6.log 2>&1 && \
PDDL_KNOBS=igemm_n64=3 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/ab/prof_n64_3 -o run --output-format csv -- python bench.py --steps 4 --warmup 2 > gpurun_out/ab/prof.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/ab/prof_def -o run --output-format csv -- python bench.py --steps 4 --warmup 2 > gpurun_out/ab/prof2.log 2>&1
rc=$?
tail -2 gpurun_out/ab/n64test.log gpurun_out/ab/kerneltests.log
grep -h '"value"' gpurun_out/ab/bench_*.log | cut -c1-200
exit $rc
