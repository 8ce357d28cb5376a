#!/bin/bash
# Calibrate the HBM byte counters (WRITE_SIZE / FETCH_SIZE) on kernels with known traffic.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/calib
S4=1024,14,256,1024,1,1,0
pass() { local tag=$1; shift; local P=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc $P -d gpurun_out/calib/$tag -o run --output-format csv -- "$@" > gpurun_out/calib/$tag.log 2>&1; }
true && \
pass sp_w WRITE_SIZE ./bench/micro/store_pattern && pass sp_f FETCH_SIZE ./bench/micro/store_pattern && \
pass fwd_rd_w WRITE_SIZE python scripts/kprobe.py --op fwd --shape $S4 --iters 5 && \
pass fwd_st_w WRITE_SIZE python scripts/kprobe.py --op fwd --shape $S4 --iters 5 --set igemm_rd=0 && \
pass fwdres_st_w WRITE_SIZE python scripts/kprobe.py --op fwdres --shape $S4 --iters 5 --set igemm_rd=0 && \
pass fwdres_st_f FETCH_SIZE python scripts/kprobe.py --op fwdres --shape $S4 --iters 5 --set igemm_rd=0
