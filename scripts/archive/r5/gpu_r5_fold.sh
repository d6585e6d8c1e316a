# Round 5: BN applies folded into the consumer convs' operand loads (ResNet-50 bn1 / bn2) - kernel and
# model tests, ps data-plane tests, then the ResNet-50 A/B (fold on / off via the test hook) and the
# ps apply stream variants.
set -o pipefail
O=gpurun_out/${1:-r5fold}
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_resnet.py tests/test_igemm_gpu.py tests/test_norm_gpu.py > $O/pytest_r50.log 2>&1
rc=$?; tail -3 $O/pytest_r50.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest_r50.log | head -30; exit $rc; }
for r in 1 2; do
  for f in 1 0; do
    DTFE_R5_FOLD=$f timeout -k 10 300 python3 bench.py --model resnet50 --steps 20 --warmup 5 > $O/r50_f${f}_$r.log 2>&1 || { tail -5 $O/r50_f${f}_$r.log; exit 1; }
    echo "r50 fold=$f $r $(grep -o '"value": [0-9.]*' $O/r50_f${f}_$r.log) $(grep -o '"ms_per_step": [0-9.]*' $O/r50_f${f}_$r.log)"
  done
done
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_cluster_gpu.py > $O/pytest_cluster.log 2>&1
rc=$?; tail -3 $O/pytest_cluster.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest_cluster.log | head -30; exit $rc; }
for st in normal high cu32 cu64 normal high; do
  timeout -k 10 240 python3 bench.py --mode ps --gpus 1 --steps 200 --warmup 20 --ps_stream $st > $O/ps11_$st.log 2>&1 || { tail -5 $O/ps11_$st.log; exit 1; }
  echo "ps11 $st $(grep -o '"value": [0-9.]*' $O/ps11_$st.log) $(grep -o '"ms_per_step": [0-9.]*' $O/ps11_$st.log)"
done
for st in normal high; do
  timeout -k 10 240 python3 bench.py --mode ps --gpus 2 --steps 200 --warmup 20 --ps_stream $st > $O/ps12_$st.log 2>&1 || { tail -5 $O/ps12_$st.log; exit 1; }
  echo "ps12 $st $(grep -o '"value": [0-9.]*' $O/ps12_$st.log) $(grep -o '"ms_per_step": [0-9.]*' $O/ps12_$st.log) $(grep -o '"ps_refreshed_ranges": [0-9]*' $O/ps12_$st.log)"
done
timeout -k 10 200 python3 bench/cnn_kernels.py --iters 30 > $O/cnn_kernels.txt 2>&1 || { tail -5 $O/cnn_kernels.txt; exit 1; }
cat $O/cnn_kernels.txt
timeout -k 10 300 python3 bench/ipc_interference.py --reps 40 > $O/ipc_caps.txt 2>&1 || { tail -5 $O/ipc_caps.txt; exit 1; }
grep "grid cap" $O/ipc_caps.txt
timeout -k 10 200 python3 bench/write_roofline.py > $O/write_roofline.txt 2>&1 || { tail -5 $O/write_roofline.txt; exit 1; }
cat $O/write_roofline.txt
