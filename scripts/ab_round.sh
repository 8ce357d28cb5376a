# ad-hoc GPU session: end-of-round check -- the whole GPU suite, smoke, then the default bench
# twice and b1024 once (final numbers for README / BASELINE)
set -o pipefail
mkdir -p gpurun_out/fin
export TMPDIR=/tmp
bash scripts/gpu_round.sh gputests smoke && \
timeout -k 10 300 python bench.py > gpurun_out/fin/d1.log 2>&1 && \
timeout -k 10 300 python bench.py --batch 1024 > gpurun_out/fin/b1024.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/fin/d2.log 2>&1
rc=$?
for f in gpurun_out/fin/*.log; do echo "$f $(grep -ho '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"peak_mem_gb": [0-9.]*' $f | tr '\n' ' ')"; done
exit $rc
