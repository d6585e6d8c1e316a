#!/bin/bash
# Round 6: training steps per hipGraph replay (bench.py --steps_per_graph) A/B, driver shape.
set -o pipefail
O=gpurun_out/r6spg; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_bench_gpu.py > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
row() { local tag=$1; shift; timeout -k 10 200 python3 bench.py "$@" > $O/$tag.log 2>&1 || { tail -3 $O/$tag.log; exit 1; }
  echo "$tag $(tail -1 $O/$tag.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("median_window_ms_per_step"), d["config"].get("steps_per_graph"))')"; }
for r in 1 2; do for S in 1 2 4 10; do row cnn_s${S}_$r --steps 20 --warmup 5 --steps_per_graph $S || exit 1; done; done
for S in 1 4; do row r20_s$S --model resnet20 --steps 20 --warmup 5 --steps_per_graph $S || exit 1; done
row cnn_pw0_s4 --steps 20 --warmup 5 --prewarm_ms 0 --steps_per_graph 4 || exit 1
row cnn_x2_s4 --gpus 2 --backend gloo --comm ipc --steps 20 --warmup 5 --steps_per_graph 4 || exit 1
for S in 1 4; do timeout -k 10 150 python bench/ref_models.py --steps 400 --warmup 40 --steps_per_graph $S 2>&1 | grep model || exit 1; done
