# ResNet-50 all-taps 3x3 weight-gradient (igemm_wgrad3) split target sweep, alternating on one box; GPU tests first
set -o pipefail
O=gpurun_out/r4w3
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_resnet.py tests/test_igemm_gpu.py tests/test_igemm_tiles_gpu.py -m gpu > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -30; exit $rc; }
for r in 1 2 3; do
  for t in 256 192 128; do
    AB_W3TARGET=$t timeout -k 10 300 python3 bench.py --model resnet50 --steps 20 --warmup 5 > $O/r50_${t}_$r.log 2>&1 || { tail -5 $O/r50_${t}_$r.log; exit 1; }
    echo "w3target=$t $(grep -o '"value": [0-9.]*' $O/r50_${t}_$r.log) $(grep -o '"ms_per_step": [0-9.]*' $O/r50_${t}_$r.log)"
  done
done
