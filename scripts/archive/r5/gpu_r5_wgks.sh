# Round 5: shortcut gradient in the dgrad epilogue + k-group split persistent wgrad (ResNet-20)
set -o pipefail
O=gpurun_out/r5wgks
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_imgconv.py tests/test_resnet.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -30; exit $rc; }
for d in 0 1; do
  echo "== iwk=$d"
  DTFE_DIAG=iwk=$d timeout -k 10 120 python3 bench/resnet20_kernels.py --only "wgrad,conv1 dgrad,shortcut" > $O/k$d.txt 2>&1 || { tail -5 $O/k$d.txt; exit 1; }
  grep -v amdgpu.ids $O/k$d.txt
done
for rep in 1 2; do
for d in 0 1; do
  DTFE_DIAG=iwk=$d timeout -k 10 200 python3 bench.py --model resnet20 --steps 20 --warmup 5 > $O/bench$d.log 2>&1 || { tail -5 $O/bench$d.log; exit 1; }
  echo "iwk=$d $(grep -o '"ms_per_step": [0-9.]*' $O/bench$d.log)"
done; done
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 > $O/cnn.log 2>&1 || { tail -5 $O/cnn.log; exit 1; }
echo "cnn $(grep -o '"ms_per_step": [0-9.]*' $O/cnn.log)"
