set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_runtime.py -v --timeout 200 --timeout-method thread -k "hung or watchdog or comm_proxy or init_rank" > gpurun_out/rt.log 2>&1
rc=$?; grep -E "PASS|FAIL|passed|failed|Error" gpurun_out/rt.log | tail -12
[ $rc -eq 0 ] || exit $rc
bash scripts/r4_comm_proxy.sh
