# fused optimizer: nontemporal fp32 master / slot stores (new) vs plain stores (DTFE_KERNEL_LIB = HEAD's optim.hip), CNN + ResNet-50
set -o pipefail
O=gpurun_out/r4nt
mkdir -p $O
AB=$PWD/distributed-tensorflow-examples_amd/_C/ab/libdtfe_kernels.so
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_kernels_gpu.py -k "optim or adam or apply" tests/test_mnist_cnn_gpu.py > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -30; exit $rc; }
for r in 1 2 3; do
  timeout -k 10 120 python3 bench.py --steps 300 --warmup 30 > $O/cnn_new_$r.log 2>&1 || exit 1
  DTFE_KERNEL_LIB=$AB timeout -k 10 120 python3 bench.py --steps 300 --warmup 30 > $O/cnn_old_$r.log 2>&1 || exit 1
  echo "cnn new $(grep -o '"ms_per_step": [0-9.]*' $O/cnn_new_$r.log)  old $(grep -o '"ms_per_step": [0-9.]*' $O/cnn_old_$r.log)"
done
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --model resnet50 --steps 20 --warmup 5 > $O/r50_new_$r.log 2>&1 || exit 1
  DTFE_KERNEL_LIB=$AB timeout -k 10 300 python3 bench.py --model resnet50 --steps 20 --warmup 5 > $O/r50_old_$r.log 2>&1 || exit 1
  echo "r50 new $(grep -o '"ms_per_step": [0-9.]*' $O/r50_new_$r.log)  old $(grep -o '"ms_per_step": [0-9.]*' $O/r50_old_$r.log)"
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 bench.py --steps 30 --warmup 5 --prewarm_ms 0 > $O/prof.log 2>&1 || exit 1
f=$(find $O/prof -name "*kernel_trace.csv" | head -1); python3 scripts/timeline.py "$f" conv1c_fwd > $O/cnn_timeline.txt; tail -14 $O/cnn_timeline.txt
