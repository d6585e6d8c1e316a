# wgrad3 gated to 64->64, optimizer tile batching, PS profiling exit: tests, ResNet-50 (+ BN-backward
# epilogue fusion A/B), CNN (+ conv2-wgrad-after-dgrad A/B), PS kernel trace, implicit-GEMM PMC passes.
set -o pipefail
O=gpurun_out/r3d
mkdir -p $O
timeout -k 10 700 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_igemm_tiles_gpu.py tests/test_resnet.py tests/test_mnist_cnn_gpu.py tests/test_kernels_gpu.py tests/test_norm_gpu.py tests/test_cluster_gpu.py > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -20; exit $rc; }
r50() { grep '^{' $1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["last_loss"])'; }
cnn() { grep '^{' $1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["median_window_ms_per_step"])'; }
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --model resnet50 --steps 20 --warmup 5 > $O/r50_$i.log 2>&1 || exit 1
  echo "r50 $(r50 $O/r50_$i.log)"
  DTFE_BN_BWD_FUSE=1 timeout -k 10 300 python3 bench.py --model resnet50 --steps 20 --warmup 5 > $O/r50bb_$i.log 2>&1 || exit 1
  echo "r50 bnbwdfuse $(r50 $O/r50bb_$i.log)"
done
for i in 1 2; do
  timeout -k 10 200 python3 bench.py --steps 200 --warmup 20 > $O/cnn_$i.log 2>&1 || exit 1
  echo "cnn $(cnn $O/cnn_$i.log)"
  DTFE_CNN_C2_AFTER=1 timeout -k 10 200 python3 bench.py --steps 200 --warmup 20 > $O/cnnA_$i.log 2>&1 || exit 1
  echo "cnn c2after $(cnn $O/cnnA_$i.log)"
done
timeout -k 10 200 python3 bench.py --mode ps --gpus 1 --steps 200 --warmup 20 > $O/ps.log 2>&1 || exit 1
echo "ps $(grep '^{' $O/ps.log | cut -c1-220)"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
DTFE_PROFILE_EXIT=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_ps -o run -- python3 bench.py --mode ps --gpus 1 --steps 40 --warmup 10 > $O/prof_ps.log 2>&1 || exit 1
find $O/prof_ps -name "*kernel_trace.csv" | head -5
bash scripts/pmc.sh r3d_convs -- python3 bench/resnet50_convs.py --batch 256 --reps 2 --no-torch > $O/pmc.txt 2>&1 || { tail -5 $O/pmc.txt; exit 1; }
grep -E "^kernel|igemm" $O/pmc.txt | cut -c1-300
