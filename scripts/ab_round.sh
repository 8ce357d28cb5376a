# ad-hoc GPU session (edited per experiment); every step bounded, chained with &&
set -o pipefail
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
b() { local n=$1; shift; timeout -k 10 300 python bench.py "$@" > gpurun_out/ab/$n.log 2>&1; }
p() { local n=$1; shift; timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/ab/prof_$n -o run --output-format csv -- python bench.py --steps 4 --warmup 2 "$@" > gpurun_out/ab/prof_$n.log 2>&1; }
PDDL_REHEARSE=1 b reh_hvd --gpus 2 --batch 256 --steps 5 --warmup 2 && \
PDDL_REHEARSE=1 b reh_mir --gpus 2 --strategy mirrored --batch 256 --steps 5 --warmup 2 && \
b bntrain --bn-mode train --steps 10 --warmup 3 && \
b fp32 --precision fp32 --steps 10 --warmup 3 && \
b c160 --batch 256 --image-size 160 --steps 20 --warmup 5 && \
b c244 --batch 256 --image-size 244 --steps 20 --warmup 5 && \
b c224 --batch 256 --steps 20 --warmup 5 && \
p c160 --batch 256 --image-size 160 && p c244 --batch 256 --image-size 244
rc=$?
grep -h '"value"' gpurun_out/ab/*.log | cut -c1-260
exit $rc
