# ad-hoc GPU session (edited per experiment); every step bounded, chained with &&
# current: per-GPU batch plateau (b512 .. b1024, alternating)
set -o pipefail
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
b() { local n=$1; shift; timeout -k 10 300 python bench.py "$@" > gpurun_out/ab/$n.log 2>&1; }
p() { local n=$1; shift; timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ab/prof_$n -o run --output-format csv -- python bench.py --steps 4 --warmup 2 "$@" > gpurun_out/ab/prof_$n.log 2>&1; }
true && \
b b512 --batch 512 && b b768 --batch 768 && b b1024 --batch 1024 && b b896 --batch 896 && b b640 --batch 640 && \
b b1024b --batch 1024 && b b512b --batch 512 && b b768b --batch 768
rc=$?
tail -n 3 gpurun_out/ab/tests.log
for f in gpurun_out/ab/b*.log; do echo "$f $(grep -h '"value"' $f | cut -c100-160)"; done
exit $rc
