# Round-4: the pruned CNN schedule, fp32 CNN path, evaluate, CLI allreduce schedule, split-K determinism;
# then the driver-shaped bench.
set -o pipefail
O=gpurun_out/r4cnn
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_mnist_cnn_gpu.py tests/test_rccl_gpu.py tests/test_cluster_gpu.py tests/test_kernels_gpu.py \
  -k "cnn or splitk" > $O/pytest.log 2>&1
rc=$?; tail -5 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -30; exit $rc; }
timeout -k 10 180 python3 bench.py --steps 20 --warmup 5 > $O/b_driver.log 2>&1 && tail -1 $O/b_driver.log | cut -c1-200
