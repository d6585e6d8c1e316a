#!/bin/bash
# Round 6: GAN / autoencoder step traces after the fusions (kernel times per launch).
set -o pipefail
O=gpurun_out/r6rt2; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for m in gan encoder; do
  timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/$m -o run -- \
    python $GRAFT_REPO_ROOT/bench/ref_models.py --models $m --steps 30 --warmup 10 > $GRAFT_REPO_ROOT/$O/$m.log 2>&1 || exit 1
done
cd $GRAFT_REPO_ROOT && python scripts/timeline.py $O/gan/run_kernel_trace.csv uniform_fill 25
