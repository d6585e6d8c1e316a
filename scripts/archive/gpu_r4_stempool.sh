# ResNet-50 stem: BN + ReLU + max pool fused (bn_relu_pool3) vs bn_apply + maxpool3_fwd, alternating on one box
set -o pipefail
O=gpurun_out/r4stem
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_norm_gpu.py tests/test_resnet.py -m gpu > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -30; exit $rc; }
for r in 1 2 3; do
  for v in 0 1; do
    AB_NOFUSE=$v timeout -k 10 300 python3 bench.py --model resnet50 --steps 20 --warmup 5 > $O/r50_${v}_$r.log 2>&1 || { tail -5 $O/r50_${v}_$r.log; exit 1; }
    echo "nofuse=$v $(grep -o '"value": [0-9.]*' $O/r50_${v}_$r.log) $(grep -o '"ms_per_step": [0-9.]*' $O/r50_${v}_$r.log)"
  done
done
