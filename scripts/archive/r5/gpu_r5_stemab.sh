# Round 5: stem changes - numerics + ResNet-20 step (3 reps) + CNN step
set -o pipefail
O=gpurun_out/r5stemab
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_imgconv.py tests/test_resnet.py tests/test_mnist_cnn_gpu.py tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -30; exit $rc; }
for rep in 1 2 3; do
  timeout -k 10 200 python3 bench.py --model resnet20 --steps 20 --warmup 5 > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
  echo "r20 $(grep -o '"value": [0-9.]*' $O/b.log) $(grep -o '"ms_per_step": [0-9.]*' $O/b.log)"
done
timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 > $O/c.log 2>&1 || { tail -5 $O/c.log; exit 1; }
echo "cnn $(grep -o '"ms_per_step": [0-9.]*' $O/c.log)"
