#!/bin/bash
# Round 6: CNN step timeline of the final tree (4 steps per hipGraph replay).
set -o pipefail
O=gpurun_out/r6tl; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/cnn -o run -- \
  python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 > $GRAFT_REPO_ROOT/$O/cnn.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT
for k in 40 41 42 43; do python3 scripts/timeline.py $O/cnn/run_kernel_trace.csv conv1c_fwd $k | tail -4; done
