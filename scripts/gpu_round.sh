#!/bin/bash
# One GPU session: kernel tests -> engine tests -> smoke -> bench.  Stops at the first
# GPU fault / abort / timeout (exit codes other than 0 = pass and 1 = test failure).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name" | tee -a gpurun_out/steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/steps.log
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
for s in "$@"; do
  case $s in
    kernels) step kernels 600 python -m pytest tests/test_gpu_kernels.py -x -q ;;
    engine)  step engine 600 python -m pytest tests/test_gpu_engine.py -x -q ;;
    gputests) step gputests 900 python -m pytest tests -m gpu -x -q ;;
    runtime) step runtime 600 python -u -m pytest tests/test_gpu_runtime.py -x -v --timeout 300 --timeout-method thread ;;
    multirank) step multirank 600 python -u -m pytest tests/test_gpu_multirank.py -x -v -s --timeout 400 --timeout-method thread ;;
    psrt)    step psrt 600 python -u -m pytest tests/test_gpu_runtime.py -x -v -k parameter_server --timeout 400 --timeout-method thread ;;
    psbench) step psbench32 300 env PDDL_REHEARSE=1 python bench.py --gpus 3 --strategy ps --ps 1 --batch 32 --steps 60 &&
             step psbench256 300 env PDDL_REHEARSE=1 python bench.py --gpus 3 --strategy ps --ps 1 --batch 256 --steps 24 ;;
    smoke)   step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench)   step bench 600 python bench.py --steps 20 --warmup 5 ;;
    bench256) step bench256 600 python bench.py --steps 20 --warmup 5 --batch 256 ;;
    benchg) step benchg 600 python bench.py --steps 20 --warmup 5 --graph 1 ;;
    benchnb) step benchnb 600 env PDDL_BITMASK=0 python bench.py --steps 20 --warmup 5 ;;
    bench64) step bench64 600 python bench.py --steps 20 --warmup 5 --batch 64 ;;
    kbench)  step kbench 600 python bench/kernels.py --json gpurun_out/kbench.json ;;
    pmc)     step pmc 600 rocprofv3 -i bench/pmc.txt --kernel-trace -d gpurun_out/pmc -o run --output-format csv -- python bench/kernels.py --rounds 1 ;;
    counters) step counters 120 rocprofv3 -L ;;
    prof)    step prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 6 --warmup 3 ;;
  esac
done
