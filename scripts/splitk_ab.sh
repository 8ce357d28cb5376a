#!/bin/bash
# Split-K A/B at the reference's small per-replica batches: kernel tests, then
# bench.py with the heuristic vs PDDL_KNOBS=igemm_splitk=0 at b32/224, b256/160 and b1024/224,
# then a kernel trace of the b32 and b256/160 steps for the per-layer breakdown.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -3 "gpurun_out/$name.log" | cut -c1-400
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
[ "${SKIP_TESTS:-0}" = 1 ] || run ktests 600 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 300 --timeout-method thread -k "splitk or igemm"
for cfg in "32 224 60 10" "256 160 30 5" "1024 224 20 5"; do
  set -- $cfg
  run "b$1_s$2_split" 300 python bench.py --batch $1 --image-size $2 --steps $3 --warmup $4
  run "b$1_s$2_nosplit" 300 env PDDL_KNOBS=igemm_splitk=0 python bench.py --batch $1 --image-size $2 --steps $3 --warmup $4
done
run "b32_wg512" 300 env PDDL_KNOBS=wgrad8_min_rows=512 python bench.py --batch 32 --steps 60 --warmup 10
run "b32_wg256" 300 env PDDL_KNOBS=wgrad8_min_rows=256 python bench.py --batch 32 --steps 60 --warmup 10
run "b256_s160_wg512" 300 env PDDL_KNOBS=wgrad8_min_rows=512 python bench.py --batch 256 --image-size 160 --steps 30 --warmup 5
run "b32_graph_split" 300 python bench.py --batch 32 --steps 100 --warmup 10 --graph 1
run "b32_graph_nosplit" 300 env PDDL_KNOBS=igemm_splitk=0 python bench.py --batch 32 --steps 100 --warmup 10 --graph 1
[ "${TRACE:-1}" = 1 ] || exit 0
run prof_b32 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_b32 -o run --output-format csv -- python bench.py --batch 32 --steps 6 --warmup 3
run prof_b32_nosplit 300 env PDDL_KNOBS=igemm_splitk=0 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_b32_nosplit -o run --output-format csv -- python bench.py --batch 32 --steps 6 --warmup 3
run prof_b256_160_nosplit 300 env PDDL_KNOBS=igemm_splitk=0 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_b256_160_nosplit -o run --output-format csv -- python bench.py --batch 256 --image-size 160 --steps 6 --warmup 3
run prof_b256_160 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_b256_160 -o run --output-format csv -- python bench.py --batch 256 --image-size 160 --steps 6 --warmup 3
