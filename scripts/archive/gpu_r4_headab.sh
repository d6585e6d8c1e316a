set -e
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "head" tests/test_mnist_cnn_gpu.py > gpurun_out/abhead_tests.log 2>&1
for r in 0 1 2; do
  for v in 0 1; do
    AB_NOPARTS=$v timeout -k 10 120 python bench.py --steps 300 --warmup 30 | sed "s/^/noparts=$v /" >> gpurun_out/abhead.log
  done
done
