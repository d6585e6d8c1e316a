# Round-4: ResNet-50 backward capture order (dgrad before wgrad at each fork): tests, bench, timeline stalls
set -o pipefail
O=gpurun_out/r4r50order
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_resnet.py -m gpu > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -30; exit $rc; }
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --model resnet50 --steps 20 --warmup 5 > $O/r50_$r.log 2>&1 || { tail -5 $O/r50_$r.log; exit 1; }
  echo "r50 $(grep -o '"value": [0-9.]*' $O/r50_$r.log) $(grep -o '"ms_per_step": [0-9.]*' $O/r50_$r.log)"
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 bench.py --model resnet50 --steps 6 --warmup 4 > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
f=$(find $O/prof -name "*kernel_trace.csv" | head -1); python3 scripts/timeline.py "$f" stem_fwd > $O/timeline.txt; tail -3 $O/timeline.txt
