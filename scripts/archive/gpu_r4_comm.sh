# Round-4: CNN/cluster GPU tests (incl. the crash -> watchdog test), fc-Adam side-stream A/B,
# IPC all-reduce interference on the overlapped conv kernels, ResNet-50 --bucket_mb sweep (W=2 on one GPU).
set -o pipefail
O=gpurun_out/r4comm
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_mnist_cnn_gpu.py tests/test_rccl_gpu.py tests/test_cluster_gpu.py > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -30; exit $rc; }
for r in 1 2; do
  for v in 0 1; do
    DTFE_CNN_FC_ADAM_SIDE=$v timeout -k 10 180 python3 bench.py --steps 200 --warmup 20 > $O/cnn1_side${v}_$r.log 2>&1 || exit 1
    echo "N=1 side=$v r$r $(grep -o '"ms_per_step": [0-9.]*' $O/cnn1_side${v}_$r.log)"
    DTFE_CNN_FC_ADAM_SIDE=$v timeout -k 10 240 python3 bench.py --gpus 2 --backend gloo --comm ipc --steps 100 --warmup 20 > $O/cnn2_side${v}_$r.log 2>&1 || exit 1
    echo "N=2(shared GPU) side=$v r$r $(grep -o '"ms_per_step": [0-9.]*' $O/cnn2_side${v}_$r.log)"
  done
done
timeout -k 10 240 python3 bench/ipc_interference.py > $O/ipc_interference.txt 2>&1 || { tail -5 $O/ipc_interference.txt; exit 1; }
cat $O/ipc_interference.txt | grep -v amdgpu.ids
for mb in 2 4 8 16 32; do
  timeout -k 10 280 python3 bench.py --model resnet50 --gpus 2 --backend gloo --comm ipc --bucket_mb $mb --steps 10 --warmup 3 > $O/r50_bucket$mb.log 2>&1 || { tail -5 $O/r50_bucket$mb.log; exit 1; }
  echo "bucket_mb=$mb $(grep -o '"ms_per_step": [0-9.]*' $O/r50_bucket$mb.log)"
done
