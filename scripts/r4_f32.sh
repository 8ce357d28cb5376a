#!/bin/bash
# fp32 conv kernels: per-shape micro-bench (64x64 vs 128x128 kernels) + a kernel trace of the fp32 step
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/f32
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u bench/f32.py --variants 0,2 > $OUT/micro.txt 2>&1 || exit $?
timeout -k 10 200 python bench.py --precision fp32 --batch 256 --steps 6 --warmup 2 > $OUT/b.json 2> $OUT/b.err || exit $?
cat $OUT/b.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --precision fp32 --batch 256 --steps 2 --warmup 1 > $OUT/prof.log 2>&1
