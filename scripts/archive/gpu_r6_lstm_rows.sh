#!/bin/bash
# Round 6: the LSTM head on B/16 workgroups (dense_head row-split form) - tests, ref bench, step timeline.
set -o pipefail
O=gpurun_out/r6lr; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_dense_head.py tests/test_models_gpu.py -k "dense_head or lstm" \
  > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/tests.log | head; exit $rc; }
for i in 1 2 3; do timeout -k 10 120 python bench/ref_models.py --models lstm --steps 400 --warmup 40 || exit 1; done 2>&1 | grep model
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/lstm -o run -- \
  python $GRAFT_REPO_ROOT/bench/ref_models.py --models lstm --steps 30 --warmup 10 > $GRAFT_REPO_ROOT/$O/lstm.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && python scripts/timeline.py $O/lstm/run_kernel_trace.csv lstm_split_fwd 25
