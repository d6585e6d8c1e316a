# Round 6: ResNet-50 - where the per-step copyBuffer dispatches come from, PMC of the 56x56 1x1 convs next to the
# HBM fill / copy rows (bench/write_roofline.py).  Counter names are checked against rocprofv3 -L first.
set -o pipefail
O=gpurun_out/${1:-r6r50}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --model resnet50 --steps 8 --warmup 3 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$O/prof.log; exit 1; }
cd $GRAFT_REPO_ROOT
python3 scripts/copybuf_origin.py $(ls $O/prof/run_kernel_trace.csv) stem_fwd --steps 3 > $O/copybuf.txt && cat $O/copybuf.txt
timeout -k 10 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
want="TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum TCP_TCC_WRITE_REQ_sum TCP_TCC_READ_REQ_sum SQ_WAIT_ANY SQ_INSTS_VMEM_WR"
for c in $want; do grep -q "${c%_sum}" $O/counters.txt && echo "have $c" || echo "MISSING $c"; done
python3 bench/write_roofline.py --reps 20 > $O/roof.log 2>&1 || { tail -5 $O/roof.log; exit 1; }
cat $O/roof.log
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE" \
           "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_sum" \
           "TCC_HIT_sum TCC_MISS_sum TCP_TCC_WRITE_REQ_sum TCP_TCC_READ_REQ_sum"; do
  i=$((i+1))
  ok=1; for c in $set; do grep -q "${c%_sum}" $O/counters.txt || ok=0; done
  [ $ok -eq 1 ] || { echo "skip pass $i (counter missing)"; continue; }
  timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d $O/pmc_$i -o run -- python3 bench/write_roofline.py --reps 5 > $O/pmc_$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $O/pmc_$i.log; exit 1; }
done
python3 scripts/pmc_summary.py "$O/pmc_*/**/*counter_collection.csv" > $O/pmc_summary.csv
cat $O/pmc_summary.csv
