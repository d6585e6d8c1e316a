#!/bin/bash
# Round 6: GAN discriminator head in one launch, autoencoder MSE without memset + in-place captured batch.
set -o pipefail
O=gpurun_out/r6rf; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_models_gpu.py \
  > $O/tests.log 2>&1; rc=$?; tail -4 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do timeout -k 10 150 python bench/ref_models.py --steps 400 --warmup 40 || exit 1; done \
  > $O/bench.txt 2>&1; rc=$?; cat $O/bench.txt; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
for m in gan encoder; do
  timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/$m -o run -- \
    python $GRAFT_REPO_ROOT/bench/ref_models.py --models $m --steps 30 --warmup 10 > $GRAFT_REPO_ROOT/$O/$m.log 2>&1 || exit 1
done
