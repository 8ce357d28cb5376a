# ad-hoc GPU session: the K = 64 residual-gradient dgrad (conv2_block{2,3} c1 dgrad) on the persistent ring
# kernel vs the per-tile kernel, standalone (scripts/kprobe.py), b1024 and b2560 shapes, alternating
set -o pipefail
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
k() { timeout -k 10 120 python scripts/kprobe.py --op dgrad_add --iters 20 "$@" >> gpurun_out/ab/kp.log 2>&1; }
k --shape 1024,56,256,64,1,1,0 --set igemm_pk=2 && k --shape 1024,56,256,64,1,1,0 --set igemm_pk=0 && \
k --shape 1024,56,256,64,1,1,0 --set igemm_pk=2 && k --shape 1024,56,256,64,1,1,0 --set igemm_pk=0 && \
k --shape 2560,56,256,64,1,1,0 --set igemm_pk=2 && k --shape 2560,56,256,64,1,1,0 --set igemm_pk=0 && \
k --shape 1024,28,512,128,1,1,0 --set igemm_pk=2 && k --shape 1024,28,512,128,1,1,0 --set igemm_pk=0
rc=$?
grep '"op"' gpurun_out/ab/kp.log
exit $rc
