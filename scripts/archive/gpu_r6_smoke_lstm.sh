#!/bin/bash
# Round 6: the strengthened smoke() and the LSTM step timeline after the staging fold.
set -o pipefail
O=gpurun_out/r6sl; mkdir -p $O
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; tail -2 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/lstm -o run -- \
  python $GRAFT_REPO_ROOT/bench/ref_models.py --models lstm --steps 30 --warmup 10 > $GRAFT_REPO_ROOT/$O/lstm.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && python scripts/timeline.py $O/lstm/run_kernel_trace.csv lstm_split_fwd 25
