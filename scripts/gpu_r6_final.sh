# Round 6 final check on a fresh box: full GPU suite, smoke, every bench row (incl. async-PS and 2-rank rehearsals)
set -o pipefail
O=gpurun_out/${1:-r6final}
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -30; exit $rc; }
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
row() {  # tag, then bench.py args
  local tag=$1; shift
  timeout -k 10 300 python3 bench.py "$@" > $O/$tag.log 2>&1 || { tail -5 $O/$tag.log; exit 1; }
  echo "$tag $(tail -1 $O/$tag.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d.get("replicas_identical", ""))')"
}
row cnn_pw150_a --steps 20 --warmup 5
row cnn_pw150_b --steps 20 --warmup 5
row cnn_pw0 --steps 20 --warmup 5 --prewarm_ms 0
row cnn_fp32 --dtype fp32 --steps 20 --warmup 5
row r20 --model resnet20 --steps 20 --warmup 5
row r50 --model resnet50 --steps 20 --warmup 5
row cnn_x2_ipc --gpus 2 --backend gloo --comm ipc --steps 20 --warmup 5
row r20_x2_ipc --model resnet20 --gpus 2 --backend gloo --comm ipc --steps 20 --warmup 5
row ps_1p1w --mode ps --gpus 1 --steps 200 --warmup 20
row ps_1p8w --mode ps --gpus 8 --steps 200 --warmup 20
row ps_2p8w --mode ps --gpus 8 --num_ps 2 --ps_partition_mb 4 --steps 200 --warmup 20
timeout -k 10 200 python3 bench/ref_models.py > $O/ref.log 2>&1 || { tail -5 $O/ref.log; exit 1; }
grep ms_per_step $O/ref.log
echo done
