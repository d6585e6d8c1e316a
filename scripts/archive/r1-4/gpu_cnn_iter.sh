# CNN kernel iteration: numerics tests, conv2 scaling, headline bench (all under their own time limits)
set -o pipefail
out=gpurun_out/${1:-r2h}
mkdir -p $out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_imgconv.py tests/test_mnist_cnn_gpu.py > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
timeout -k 10 120 python3 bench/conv2_scale.py > $out/conv2_scale.txt 2>&1 && cat $out/conv2_scale.txt | grep B=
timeout -k 10 200 python3 bench.py --steps 200 --warmup 20 > $out/bench.log 2>&1 && grep '^{' $out/bench.log | cut -c1-300
timeout -k 10 200 python3 bench/cnn_kernels.py > $out/cnn_kernels.txt 2>&1 && cat $out/cnn_kernels.txt
