#!/bin/bash
# Round 6: CNN deferred conv2-branch join (device-side signal to Adam, one stream join per replay) - tests + A/B.
set -o pipefail
O=gpurun_out/r6dj; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_graphs_gpu.py tests/test_mnist_cnn_gpu.py \
  > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/tests.log | head; exit $rc; }
row() { local tag=$1; shift; timeout -k 10 200 python3 bench.py "$@" > $O/$tag.log 2>&1 || { tail -3 $O/$tag.log; exit 1; }
  echo "$tag $(tail -1 $O/$tag.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("median_window_ms_per_step"), d["config"].get("join_deferred"), d["config"].get("last_loss"))')"; }
for r in 1 2 3; do
  row def_$r --steps 20 --warmup 5 || exit 1
  row nodefer_$r --steps 20 --warmup 5 --no_join_defer || exit 1
done
row pw0 --steps 20 --warmup 5 --prewarm_ms 0 || exit 1
row odd --steps 7 --warmup 3 || exit 1
