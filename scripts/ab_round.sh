# ad-hoc GPU session: kernel trace of the default configuration (b2560) for the README step breakdown
set -o pipefail
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/ab/prof_d -o run --output-format csv -- python bench.py --steps 4 --warmup 2 > gpurun_out/ab/prof_d.log 2>&1
rc=$?
grep -h '"value"' gpurun_out/ab/prof_d.log | grep -o '"value": [0-9.]*'
exit $rc
