#!/bin/bash
# Round 6: LSTM batch staging folded into the split forward launch - tests, ref_models A/B, kernel trace.
set -o pipefail
O=gpurun_out/r6lst; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_models_gpu.py -k lstm \
  > $O/tests.log 2>&1 && tail -3 $O/tests.log &&
for i in 1 2 3; do timeout -k 10 120 python bench/ref_models.py --models lstm --steps 400 --warmup 40 || exit 1; done \
  > $O/bench.txt 2>&1 && cat $O/bench.txt &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- \
  python $GRAFT_REPO_ROOT/bench/ref_models.py --models lstm --steps 50 --warmup 10 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 &&
cd $GRAFT_REPO_ROOT && python scripts/timeline.py "$(find $O/prof -name "*kernel_trace.csv" | head -1)" lstm_split_fwd \
  > $O/timeline.txt 2>&1; cat $O/timeline.txt
