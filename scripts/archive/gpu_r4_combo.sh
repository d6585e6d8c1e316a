# Round-4: (1) fused ps replies; (2) BN 1-bit ReLU mask; (3) CNN conv wgrad reduces folded into Adam.
# tests, benches (ps 1+1, ResNet-50, CNN), ps timeline, CNN + ResNet-50 kernel tables
set -o pipefail
O=gpurun_out/r4combo
mkdir -p $O
timeout -k 10 700 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_mnist_cnn_gpu.py tests/test_norm_gpu.py tests/test_igemm_gpu.py tests/test_cluster_gpu.py tests/test_resnet.py -m gpu > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -30; exit $rc; }
for i in 1 2; do
  timeout -k 10 180 python3 bench.py --steps 200 --warmup 20 > $O/cnn_$i.log 2>&1 || { tail -5 $O/cnn_$i.log; exit 1; }
  echo "cnn $(grep -o '"value": [0-9.]*' $O/cnn_$i.log) $(grep -o '"ms_per_step": [0-9.]*' $O/cnn_$i.log)"
  timeout -k 10 240 python3 bench.py --mode ps --gpus 1 --steps 200 --warmup 20 > $O/ps11_$i.log 2>&1 || { tail -5 $O/ps11_$i.log; exit 1; }
  echo "ps11 $(grep -o '"ms_per_step": [0-9.]*' $O/ps11_$i.log)"
  timeout -k 10 300 python3 bench.py --model resnet50 --steps 20 --warmup 5 > $O/r50_$i.log 2>&1 || { tail -5 $O/r50_$i.log; exit 1; }
  echo "r50 $(grep -o '"value": [0-9.]*' $O/r50_$i.log) $(grep -o '"ms_per_step": [0-9.]*' $O/r50_$i.log)"
done
timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 > $O/cnn_driver.log 2>&1 && echo "cnn driver-shaped $(grep -o '"ms_per_step": [0-9.]*' $O/cnn_driver.log)"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
DTFE_PROFILE_EXIT=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_ps -o run_%pid% -- python3 bench.py --mode ps --gpus 1 --steps 40 --warmup 10 > $O/prof_ps.log 2>&1 || { tail -5 $O/prof_ps.log; exit 1; }
python3 scripts/ps_timeline.py $O/prof_ps > $O/ps_timeline.txt 2>&1; tail -12 $O/ps_timeline.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_cnn -o run -- python3 bench.py --steps 30 --warmup 5 > $O/prof_cnn.log 2>&1 || { tail -5 $O/prof_cnn.log; exit 1; }
f=$(find $O/prof_cnn -name "*kernel_stats.csv" | head -1); python3 scripts/kstats.py "$f" > $O/cnn_kernels.txt
f=$(find $O/prof_cnn -name "*kernel_trace.csv" | head -1); python3 scripts/timeline.py "$f" conv1c_fwd > $O/cnn_timeline.txt; cat $O/cnn_timeline.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_r50 -o run -- python3 bench.py --model resnet50 --steps 8 --warmup 5 > $O/prof_r50.log 2>&1 || { tail -5 $O/prof_r50.log; exit 1; }
f=$(find $O/prof_r50 -name "*kernel_stats.csv" | head -1); python3 scripts/kstats.py "$f" > $O/r50_kernels.txt; head -24 $O/r50_kernels.txt
