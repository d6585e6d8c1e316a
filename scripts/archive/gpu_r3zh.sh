# Validate the conv1 weight-gradient grid default (320): CNN GPU tests + default bench + smoke.
set -o pipefail
O=gpurun_out/r3zh
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_imgconv.py tests/test_mnist_cnn_gpu.py tests/test_kernels_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -1 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -20; exit $rc; }
timeout -k 10 180 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && tail -1 $O/smoke.log &&
timeout -k 10 180 python3 bench.py > $O/b_default.log 2>&1 && tail -1 $O/b_default.log | cut -c1-200 &&
timeout -k 10 180 python3 bench.py --steps 20 --warmup 5 > $O/b_driver.log 2>&1 && tail -1 $O/b_driver.log | cut -c1-200
