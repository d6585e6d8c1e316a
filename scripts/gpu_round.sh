set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/ -m gpu -x -q > gpurun_out/t2.log 2>&1; echo "TEST EXIT $?" >> gpurun_out/t2.log
tail -5 gpurun_out/t2.log
for b in 128 1024; do timeout -k 10 120 python bench.py --steps 100 --warmup 10 --batch_size $b 2>&1 | grep metric; done
bash scripts/profile.sh b1024 --steps 30 --warmup 5 --batch_size 1024
