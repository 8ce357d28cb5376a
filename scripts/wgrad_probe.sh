#!/bin/bash
# wgrad8 with and without its atomic epilogue (knob +8 = timing probe), per layer shape.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for s in 256,14,256,256,3,1,1 256,7,512,512,3,1,1 256,14,1024,256,1,1,0 2560,14,256,256,3,1,1 2560,14,1024,256,1,1,0 2560,7,2048,512,1,1,0; do
  for k in 1 9; do
    timeout -k 10 120 python scripts/kprobe.py --op wgrad --shape $s --set wgrad8=$k --iters 20 || exit 1
  done
done
