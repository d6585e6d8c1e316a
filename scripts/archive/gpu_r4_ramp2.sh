# driver-shaped CNN bench (--steps 20 --warmup 5) with the default 150 ms pre-warm vs none, then the bench tests
set -e
for r in 0 1; do
  for p in 150 0; do
    timeout -k 10 120 python bench.py --steps 20 --warmup 5 --prewarm_ms $p | sed "s/^/prewarm_ms=$p /" >> gpurun_out/ramp2.log
  done
done
timeout -k 10 120 python bench.py --model resnet50 --steps 20 --warmup 5 | sed "s/^/r50 /" >> gpurun_out/ramp2.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_bench_gpu.py tests/test_cluster_gpu.py > gpurun_out/ramp2_tests.log 2>&1
