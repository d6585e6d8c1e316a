# hardware bf16 rounding (v_cvt_pk_bf16_f32) in every kernel: full GPU suite, conv table, ResNet-50 / CNN benches
set -o pipefail
O=gpurun_out/r3e
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -20; exit $rc; }
timeout -k 10 400 python3 bench/resnet50_convs.py --batch 256 --reps 10 --no-torch > $O/convs.txt 2>&1 || exit 1
grep -v amdgpu.ids $O/convs.txt
r50() { grep '^{' $1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["last_loss"])'; }
cnn() { grep '^{' $1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["median_window_ms_per_step"])'; }
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --model resnet50 --steps 20 --warmup 5 > $O/r50_$i.log 2>&1 || exit 1
  echo "r50 $(r50 $O/r50_$i.log)"
  timeout -k 10 200 python3 bench.py --steps 200 --warmup 20 > $O/cnn_$i.log 2>&1 || exit 1
  echo "cnn $(cnn $O/cnn_$i.log)"
done
