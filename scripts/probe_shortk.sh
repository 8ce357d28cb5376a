#!/bin/bash
# Short-K 1x1 layer study: per-kernel timing of variants (kprobe) + HBM / L2 counter passes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/probe
o=gpurun_out/probe/times.jsonl
: > $o
k() { timeout -k 10 60 python scripts/kprobe.py --iters 30 "$@" >> $o 2>/dev/null; }
S4=1024,14,256,1024,1,1,0
S3=1024,28,128,512,1,1,0
S2=1024,56,64,256,1,1,0
true && \
k --op fwdres --shape $S4 && k --op fwdres --shape $S4 --set igemm_rd=0 && k --op fwdres --shape $S4 --set igemm_pk=2 && \
k --op fwd --shape $S4 && k --op fwd --shape $S4 --set igemm_rd=0 && \
k --op fwdres --shape $S3 && k --op fwd --shape $S3 && \
k --op fwdres --shape $S2 && k --op fwd --shape $S2 && \
k --op fwdres --shape 1024,14,64,1024,1,1,0 && k --op fwdres --shape 1024,14,512,1024,1,1,0 && \
k --op dgrad_add --shape 1024,14,1024,256,1,1,0 && k --op dgrad_add --shape 1024,14,1024,256,1,1,0 --drop add && \
k --op dgrad_add --shape 1024,14,1024,256,1,1,0 --drop add,bits,colsum && \
for P in "FETCH_SIZE" "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_WRREQ_64B_sum"; do
  tag=$(echo $P | cut -d' ' -f1)
  timeout -s KILL 60 rocprofv3 --pmc $P -d gpurun_out/probe/pmc_$tag -o run --output-format csv -- \
    python scripts/kprobe.py --op fwdres --shape $S4 --iters 5 > gpurun_out/probe/pmc_$tag.log 2>&1 || exit 1
done
cat $o
