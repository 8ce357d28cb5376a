#!/bin/bash
# Round 4: the backward under modelled 8-GPU comm contention (bench.py --comm-proxy) on one GPU,
# with the static persistent kernels (igemm_pk ring, bwd1x1, igemm8) on vs off, plus kernel
# traces of the default build with and without the proxy (per-layer deltas).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/cp
mkdir -p $OUT
export TMPDIR=/tmp
PX="world=8,busbw=350,nch=32"
run() {   # tag, env assignments..., -- bench args...
  local tag=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  timeout -k 10 240 env "${envs[@]}" python bench.py --steps 12 --warmup 4 "$@" > $OUT/$tag.json 2> $OUT/$tag.err
  local rc=$?
  [ $rc -eq 0 ] || { echo "$tag failed rc=$rc"; tail -5 $OUT/$tag.err; return $rc; }
  python -c "import json;d=json.load(open('$OUT/$tag.json'));print('$tag', d['value'], d['ms_per_step'], d.get('comm_proxy',{}).get('modelled_ms_per_step'))" | tee -a $OUT/summary.txt
}
run base X=1 -- && \
run proxy X=1 -- --comm-proxy $PX && \
run base_static_off PDDL_KNOBS=igemm_pk=0,igemm8=0 PDDL_FUSE_BWD=0 -- && \
run proxy_static_off PDDL_KNOBS=igemm_pk=0,igemm8=0 PDDL_FUSE_BWD=0 -- --comm-proxy $PX && \
run proxy_nch64 X=1 -- --comm-proxy world=8,busbw=350,nch=64 && \
run proxy_pk_off PDDL_KNOBS=igemm_pk=0 -- --comm-proxy $PX && \
run base2 X=1 -- && \
run proxy2 X=1 -- --comm-proxy $PX && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_base -o run --output-format csv -- python bench.py --steps 3 --warmup 2 > $OUT/prof_base.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_proxy -o run --output-format csv -- python bench.py --steps 3 --warmup 2 --comm-proxy $PX > $OUT/prof_proxy.log 2>&1
rc=$?
cat $OUT/summary.txt
exit $rc
