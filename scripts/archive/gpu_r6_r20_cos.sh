#!/bin/bash
# Round 6: repeat the ResNet-20 bench-shape oracle test (its BN gamma cosines vary with the bn_stats atomics).
set -o pipefail
O=gpurun_out/r6cos; mkdir -p $O
for i in 1 2 3 4; do
  timeout -k 10 200 python -u -m pytest -x -q --timeout 150 --timeout-method thread -p no:cacheprovider \
    "tests/test_resnet.py::test_resnet20_bench_shaped_step_matches_autograd" > $O/run$i.log 2>&1
  echo "run $i rc=$? $(grep -E 'passed|failed' $O/run$i.log | tail -1) $(grep -o "AssertionError: .*" $O/run$i.log | head -1)"
done
