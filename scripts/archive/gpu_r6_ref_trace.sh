#!/bin/bash
# Round 6: kernel traces of the reference's three workloads (bench/ref_models.py), one model per run.
set -o pipefail
O=gpurun_out/r6ref; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for m in gan encoder lstm; do
  timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/$m -o run -- \
    python $GRAFT_REPO_ROOT/bench/ref_models.py --models $m --steps 30 --warmup 10 > $GRAFT_REPO_ROOT/$O/$m.log 2>&1 || exit 1
done
cd $GRAFT_REPO_ROOT && find $O -name "*kernel_trace.csv" | sort
