# Round 5: ResNet-20 output-BN backward statistics in conv1's data-gradient epilogue: numerics + same-box A/B
set -o pipefail
O=gpurun_out/r5bse
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_imgconv.py tests/test_resnet.py tests/test_dense_head.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -30; exit $rc; }
for rep in 1 2 3; do
for f in 1 0; do
  DTFE_R20_BSE=$f timeout -k 10 200 python3 bench.py --model resnet20 --steps 20 --warmup 5 > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
  echo "bse=$f $(grep -o '"value": [0-9.]*' $O/b.log) $(grep -o '"ms_per_step": [0-9.]*' $O/b.log)"
done; done
