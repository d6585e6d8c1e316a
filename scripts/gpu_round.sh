set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/bench1.log
timeout -k 10 600 python -m pytest tests/ -m gpu -x -q > gpurun_out/t2.log 2>&1; echo "TEST EXIT $?" >> gpurun_out/t2.log
tail -30 gpurun_out/t2.log
for b in 128 512 1024 2048; do timeout -k 10 120 python bench.py --steps 100 --warmup 10 --batch_size $b >> gpurun_out/bench1.log 2>&1 || echo "bench $b failed $?" >> gpurun_out/bench1.log; done
grep -v amdgpu.ids gpurun_out/bench1.log
