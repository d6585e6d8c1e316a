#!/bin/bash
# Round 6: default steps-per-graph (4 on one GPU) in the driver's shapes, with and without the pre-warm.
set -o pipefail
O=gpurun_out/r6spg2; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_bench_gpu.py > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
row() { local tag=$1; shift; timeout -k 10 200 python3 bench.py "$@" > $O/$tag.log 2>&1 || { tail -3 $O/$tag.log; exit 1; }
  echo "$tag $(tail -1 $O/$tag.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("median_window_ms_per_step"), d["config"].get("steps_per_graph"), d["config"]["prewarm"])')"; }
row cnn_def_a --steps 20 --warmup 5
row cnn_s1 --steps 20 --warmup 5 --steps_per_graph 1
row cnn_def_b --steps 20 --warmup 5
row cnn_pw0 --steps 20 --warmup 5 --prewarm_ms 0
row cnn_pw0_s1 --steps 20 --warmup 5 --prewarm_ms 0 --steps_per_graph 1
row cnn_odd --steps 7 --warmup 3
row cnn_fp32 --dtype fp32 --steps 20 --warmup 5
row r20 --model resnet20 --steps 20 --warmup 5
row r50 --model resnet50 --steps 20 --warmup 5
row cnn_x2 --gpus 2 --backend gloo --comm ipc --steps 20 --warmup 5
