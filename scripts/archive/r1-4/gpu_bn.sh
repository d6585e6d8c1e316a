set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_norm_gpu.py tests/test_kernels_gpu.py tests/test_resnet.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_bn.log 2>&1 &&
timeout -k 10 120 python3 bench/bn_bench.py > gpurun_out/bn_bench.log 2>&1 &&
timeout -k 10 200 python3 bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/b_r50.log 2>&1 &&
timeout -k 10 200 python3 bench.py --steps 200 --warmup 20 --no_graph > gpurun_out/b_cnn_nograph.log 2>&1 &&
timeout -k 10 200 python3 bench.py --model resnet50 --steps 20 --warmup 5 --no_graph > gpurun_out/b_r50_nograph.log 2>&1 &&
bash scripts/profile.sh r50 --model resnet50 --steps 10 --warmup 3 > gpurun_out/prof_r50.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_bn.log; cat gpurun_out/bn_bench.log; for f in gpurun_out/b_*.log; do tail -n 1 $f | cut -c1-200; done
exit $rc
