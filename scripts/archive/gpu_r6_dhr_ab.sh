#!/bin/bash
# Round 6: dense_head_rows phase ablations (DTFE_DIAG dhr=<bits>: 1 no partial slabs / ticket, 2 no logits, 4 no softmax)
set -o pipefail
O=gpurun_out/r6dhr; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for cfg in 0 1 2 4 7; do
  DTFE_DIAG=dhr=$cfg timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/d$cfg -o run -- \
    python $GRAFT_REPO_ROOT/bench/ref_models.py --models lstm --steps 30 --warmup 10 > $GRAFT_REPO_ROOT/$O/d$cfg.log 2>&1 || exit 1
  echo "dhr=$cfg $(python3 - $GRAFT_REPO_ROOT/$O/d$cfg/run_kernel_trace.csv <<'PY'
import csv, sys, statistics
r = [(int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1000 for x in csv.DictReader(open(sys.argv[1])) if "dense_head" in x["Kernel_Name"]]
print("head us median %.2f n %d" % (statistics.median(r), len(r)))
PY
)"
done
