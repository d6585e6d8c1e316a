# Round 5: BN statistics fused into the whole-image conv forward (ResNet-20): numerics + A/B
set -o pipefail
O=gpurun_out/r5imgstats
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_imgconv.py tests/test_resnet.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -30; exit $rc; }
timeout -k 10 120 python3 bench/resnet20_kernels.py --only "conv1 fwd,conv2 fwd" > $O/k.txt 2>&1 || { tail -5 $O/k.txt; exit 1; }
grep -v amdgpu.ids $O/k.txt
for rep in 1 2; do
for f in 1 0; do
  DTFE_R5_IMGSTATS=$f timeout -k 10 200 python3 bench.py --model resnet20 --steps 20 --warmup 5 > $O/bench$f.log 2>&1 || { tail -5 $O/bench$f.log; exit 1; }
  echo "fused=$f $(grep -o '"ms_per_step": [0-9.]*' $O/bench$f.log)"
done; done
