set -o pipefail
O=gpurun_out/r6final; mkdir -p $O
for i in 1 2 3; do timeout -k 10 300 python bench.py > $O/b$i.json 2>$O/b$i.err || { tail -5 $O/b$i.err; exit 1; }
python -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]);print('b2560', d['value'], d['ms_per_step'])" $O/b$i.json; done
bash scripts/layer_prof.sh $O/layers > /dev/null 2>&1 || exit 1
tail -14 $O/layers/per_layer.txt
rm -rf $O/layers/prof
