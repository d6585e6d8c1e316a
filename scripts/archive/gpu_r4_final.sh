# Round-4 final check: every GPU test, smoke(), driver-shaped benches (CNN, ps 1+1, ResNet-50), CNN + ResNet-50
# kernel tables and step timelines (profiled runs without the pre-warm so step counts stay readable)
set -o pipefail
O=gpurun_out/r4final2
mkdir -p $O
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -30; exit $rc; }
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 && tail -1 $O/smoke.log || { tail -5 $O/smoke.log; exit 1; }
for i in 1 2; do
  timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 > $O/cnn_driver_$i.log 2>&1 || { tail -5 $O/cnn_driver_$i.log; exit 1; }
  echo "cnn driver-shaped $(grep -o '"value": [0-9.]*' $O/cnn_driver_$i.log) $(grep -o '"ms_per_step": [0-9.]*' $O/cnn_driver_$i.log)"
  timeout -k 10 180 python3 bench.py --steps 300 --warmup 30 > $O/cnn_$i.log 2>&1 || { tail -5 $O/cnn_$i.log; exit 1; }
  echo "cnn 300 steps $(grep -o '"value": [0-9.]*' $O/cnn_$i.log) $(grep -o '"ms_per_step": [0-9.]*' $O/cnn_$i.log)"
  timeout -k 10 240 python3 bench.py --mode ps --gpus 1 --steps 200 --warmup 20 > $O/ps11_$i.log 2>&1 || { tail -5 $O/ps11_$i.log; exit 1; }
  echo "ps11 $(grep -o '"ms_per_step": [0-9.]*' $O/ps11_$i.log)"
  timeout -k 10 300 python3 bench.py --model resnet50 --steps 20 --warmup 5 > $O/r50_$i.log 2>&1 || { tail -5 $O/r50_$i.log; exit 1; }
  echo "r50 $(grep -o '"value": [0-9.]*' $O/r50_$i.log) $(grep -o '"ms_per_step": [0-9.]*' $O/r50_$i.log)"
done
timeout -k 10 200 python3 bench.py --model resnet20 --steps 50 --warmup 10 > $O/r20.log 2>&1 && echo "r20 $(grep -o '"value": [0-9.]*' $O/r20.log)" || { tail -5 $O/r20.log; exit 1; }
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_cnn -o run -- python3 bench.py --steps 30 --warmup 5 --prewarm_ms 0 > $O/prof_cnn.log 2>&1 || { tail -5 $O/prof_cnn.log; exit 1; }
f=$(find $O/prof_cnn -name "*kernel_stats.csv" | head -1); python3 scripts/kstats.py "$f" > $O/cnn_kernels.txt
f=$(find $O/prof_cnn -name "*kernel_trace.csv" | head -1); python3 scripts/timeline.py "$f" conv1c_fwd > $O/cnn_timeline.txt; tail -14 $O/cnn_timeline.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_r50 -o run -- python3 bench.py --model resnet50 --steps 8 --warmup 5 --prewarm_ms 0 > $O/prof_r50.log 2>&1 || { tail -5 $O/prof_r50.log; exit 1; }
f=$(find $O/prof_r50 -name "*kernel_stats.csv" | head -1); python3 scripts/kstats.py "$f" > $O/r50_kernels.txt; head -30 $O/r50_kernels.txt
