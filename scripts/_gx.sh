set -o pipefail
O=gpurun_out/r6sk3; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "splitk" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for r in 1 2; do for k in 0 1 2; do
timeout -k 10 200 env PDDL_KNOBS=igemm_sk3=$k python bench.py --batch 32 --steps 300 --warmup 30 > $O/b_$k.json 2>&1 || exit 1
python -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]);print('sk3', sys.argv[2], d['value'], d['ms_per_step'])" $O/b_$k.json $k; done; done
