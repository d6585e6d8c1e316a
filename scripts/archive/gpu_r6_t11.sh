# Round 6: fused-statistics ablation of the ResNet-20 whole-image convs + LSTM with XCD-aligned split groups
set -o pipefail
O=gpurun_out/${1:-r6t11}
mkdir -p $O
for d in "" "icr=1024" "icr=256" "icr=512"; do
  DTFE_DIAG=$d timeout -k 10 120 python3 bench/imgconv_stats_ab.py > $O/ab_$d.log 2>&1 || { tail -5 $O/ab_$d.log; exit 1; }
  grep -v amdgpu.ids $O/ab_$d.log
done
timeout -k 10 200 python3 -u -m pytest tests/test_models_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu -k lstm > $O/pytest_lstm.log 2>&1
rc=$?; tail -2 $O/pytest_lstm.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest_lstm.log | head -30; exit $rc; }
timeout -k 10 200 python3 bench/ref_models.py --models lstm > $O/lstm.log 2>&1 || { tail -5 $O/lstm.log; exit 1; }
cat $O/lstm.log
timeout -k 10 200 python3 -u -m pytest tests/test_kernels_gpu.py tests/test_mnist_cnn_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu -k "fp32" > $O/pytest32.log 2>&1
rc=$?; tail -2 $O/pytest32.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest32.log | head -30; exit $rc; }
timeout -k 10 200 python3 bench.py --dtype fp32 --steps 30 --warmup 5 > $O/cnn32.log 2>&1 || { tail -5 $O/cnn32.log; exit 1; }
tail -1 $O/cnn32.log | cut -c1-300
