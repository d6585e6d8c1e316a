# CNN kernel microbenchmarks + new numerics tests + honest stock baselines.
set -o pipefail
O=gpurun_out/r2b
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_mnist_cnn_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest_cnn.log 2>&1
rc=$?; tail -3 $O/pytest_cnn.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 bench/cnn_kernels.py --batch_size 1024 --iters 30 > $O/cnn_kernels.txt 2>&1 && cat $O/cnn_kernels.txt &&
timeout -k 10 300 python3 bench/gemm_sweep.py --iters 20 > $O/gemm_sweep.txt 2>&1 && cat $O/gemm_sweep.txt &&
timeout -k 10 200 python3 bench/stock_torch_cnn.py --steps 100 --warmup 20 --batch_size 1024 --graph > $O/stock_cnn_graph.txt 2>&1 && cat $O/stock_cnn_graph.txt &&
timeout -k 10 200 python3 bench/stock_torch_cnn.py --steps 100 --warmup 20 --batch_size 1024 --fused > $O/stock_cnn_fused.txt 2>&1 && cat $O/stock_cnn_fused.txt &&
timeout -k 10 300 python3 bench/stock_torch_resnet.py --arch resnet50 --batch_size 256 --steps 20 --warmup 5 --graph > $O/stock_r50_graph.txt 2>&1 && cat $O/stock_r50_graph.txt &&
timeout -k 10 300 python3 bench/stock_torch_resnet.py --arch resnet50 --batch_size 256 --steps 20 --warmup 5 > $O/stock_r50.txt 2>&1 && cat $O/stock_r50.txt &&
timeout -k 10 300 python3 bench/stock_torch_resnet.py --arch resnet20 --batch_size 256 --steps 50 --warmup 10 --graph > $O/stock_r20_graph.txt 2>&1 && cat $O/stock_r20_graph.txt
