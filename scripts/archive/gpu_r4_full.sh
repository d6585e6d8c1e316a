# Round-4 full check: every GPU test, smoke(), the driver-shaped CNN bench, CNN / ps / ResNet-50 benches
set -o pipefail
O=gpurun_out/r4full
mkdir -p $O
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -30; exit $rc; }
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 && tail -1 $O/smoke.log || { tail -5 $O/smoke.log; exit 1; }
timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 > $O/cnn_driver.log 2>&1 && grep '^{' $O/cnn_driver.log | cut -c1-220 || exit 1
for i in 1 2; do
  timeout -k 10 180 python3 bench.py --steps 200 --warmup 20 > $O/cnn_$i.log 2>&1 || { tail -5 $O/cnn_$i.log; exit 1; }
  echo "cnn $(grep -o '"value": [0-9.]*' $O/cnn_$i.log) $(grep -o '"ms_per_step": [0-9.]*' $O/cnn_$i.log)"
  timeout -k 10 240 python3 bench.py --mode ps --gpus 1 --steps 200 --warmup 20 > $O/ps11_$i.log 2>&1 || { tail -5 $O/ps11_$i.log; exit 1; }
  echo "ps11 $(grep -o '"ms_per_step": [0-9.]*' $O/ps11_$i.log)"
  timeout -k 10 300 python3 bench.py --model resnet50 --steps 20 --warmup 5 > $O/r50_$i.log 2>&1 || { tail -5 $O/r50_$i.log; exit 1; }
  echo "r50 $(grep -o '"value": [0-9.]*' $O/r50_$i.log) $(grep -o '"ms_per_step": [0-9.]*' $O/r50_$i.log)"
done
