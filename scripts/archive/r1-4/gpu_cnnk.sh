set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_imgconv.py tests/test_mnist_cnn_gpu.py tests/test_kernels_gpu.py tests/test_models_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_k.log 2>&1 &&
timeout -k 10 200 python3 bench.py --steps 200 --warmup 20 > gpurun_out/b_cnn.log 2>&1 &&
bash scripts/profile.sh cnn --steps 50 --warmup 10 > gpurun_out/prof_cnn.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_k.log; tail -1 gpurun_out/b_cnn.log | cut -c1-150
exit $rc
