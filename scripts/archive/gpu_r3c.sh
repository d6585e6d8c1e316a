# all-taps 3x3 weight gradient + pruned CNN schedule: tests, per-layer conv table, ResNet-50 / CNN benches,
# and a rocprofv3 kernel trace of the 1 ps + 1 worker PS step (timeline of the bucket applies).
set -o pipefail
O=gpurun_out/r3c
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_igemm_tiles_gpu.py tests/test_resnet.py tests/test_mnist_cnn_gpu.py tests/test_kernels_gpu.py > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -20; exit $rc; }
timeout -k 10 400 python3 bench/resnet50_convs.py --batch 256 --reps 10 --no-torch > $O/convs.txt 2>&1 || exit 1
grep -E "3x3 /1|totals" $O/convs.txt
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --model resnet50 --steps 20 --warmup 5 > $O/r50_$i.log 2>&1 || exit 1
  echo "r50 $(grep '^{' $O/r50_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["last_loss"])')"
  timeout -k 10 200 python3 bench.py --steps 200 --warmup 20 > $O/cnn_$i.log 2>&1 || exit 1
  echo "cnn $(grep '^{' $O/cnn_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["median_window_ms_per_step"])')"
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_ps -o run -- python3 bench.py --mode ps --gpus 1 --steps 40 --warmup 10 > $O/prof_ps.log 2>&1 || exit 1
tail -1 $O/prof_ps.log | cut -c1-200
find $O/prof_ps -name "*kernel_trace.csv" | head
