set -o pipefail
mkdir -p gpurun_out/bis
C="--data synthetic --epochs 1 --steps-per-epoch 4 --validation-steps 0 --batch-size 256 --no-save"
AMD_LOG_LEVEL=1 timeout -k 10 200 python -u imagenet-resnet50-mirror.py $C > gpurun_out/bis/m_log1.log 2>&1
echo "rc=$?"
grep -n -m 12 -i "error\|capture" gpurun_out/bis/m_log1.log | cut -c1-300
