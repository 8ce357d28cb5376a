# ad-hoc GPU session (edited per experiment); every step bounded, chained with &&
# current: persistent ring kernel on by default (selective) -> whole GPU suite + smoke, then
# b1024 / b2048 A/B against igemm_pk=0 on the same box
set -o pipefail
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
b() { local n=$1; shift; timeout -k 10 300 python bench.py "$@" > gpurun_out/ab/$n.log 2>&1; }
true && \
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/ab/gputests.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/ab/smoke.log 2>&1 && \
b pk2 --batch 1024 && PDDL_KNOBS=igemm_pk=0 b pk0 --batch 1024 && b pk2b --batch 1024 && PDDL_KNOBS=igemm_pk=0 b pk0b --batch 1024 && \
b pk2_b2048 && PDDL_KNOBS=igemm_pk=0 b pk0_b2048
rc=$?
tail -n 3 gpurun_out/ab/gputests.log; tail -2 gpurun_out/ab/smoke.log
for f in gpurun_out/ab/*.log; do echo "$f $(grep -ho '"value": [0-9.]*' $f)"; done
exit $rc
