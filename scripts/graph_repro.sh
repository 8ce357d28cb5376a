#!/bin/bash
# The standalone hipGraphLaunch reproducer (csrc/tests/graph_replay_repro.cpp) against the ROCm
# runtime it links and against the runtime torch bundles (the one in use when the round-5 fault
# was seen), one run each.   bash scripts/graph_repro.sh OUTDIR [rounds]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/graph_repro}; R=${2:-200}
mkdir -p $OUT /tmp/pddl_torch_rt
TL=$(python -c "import torch,os;print(os.path.join(os.path.dirname(torch.__file__),'lib'))")
ln -sf $TL/libamdhip64.so /tmp/pddl_torch_rt/libamdhip64.so.7
timeout -k 10 300 ./csrc/tests/graph_replay_repro.bin $R > $OUT/rocm72.txt 2>&1; echo "rocm runtime exit $?" >> $OUT/rocm72.txt
tail -2 $OUT/rocm72.txt
LD_LIBRARY_PATH=/tmp/pddl_torch_rt:$LD_LIBRARY_PATH timeout -k 10 300 ./csrc/tests/graph_replay_repro.bin $R > $OUT/torch_rt.txt 2>&1
echo "torch runtime exit $?" >> $OUT/torch_rt.txt
tail -2 $OUT/torch_rt.txt
