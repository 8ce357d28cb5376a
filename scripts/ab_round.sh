# ad-hoc GPU session (edited per experiment); every step bounded, chained with &&
# current: validation of the tree: whole GPU suite + smoke + default bench twice + b1024
set -o pipefail
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
b() { local n=$1; shift; timeout -k 10 300 python bench.py "$@" > gpurun_out/ab/$n.log 2>&1; }
true && \
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/ab/gputests.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/ab/smoke.log 2>&1 && \
b def && b def2 && b b1024 --batch 1024
rc=$?
tail -n 2 gpurun_out/ab/gputests.log; tail -1 gpurun_out/ab/smoke.log
for f in gpurun_out/ab/*.log; do echo "$f $(grep -ho '"value": [0-9.]*\|"ms_per_step": [0-9.]*' $f | tr '\n' ' ')"; done
exit $rc
