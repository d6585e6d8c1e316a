# Round 6: ResNet-50 - bench, where the per-step copyBuffer dispatches come from, PMC of the 56x56 1x1 convs
set -o pipefail
O=gpurun_out/${1:-r6r50}
mkdir -p $O
timeout -k 10 300 python3 bench.py --model resnet50 --steps 20 --warmup 5 > $O/r50.log 2>&1 || { tail -5 $O/r50.log; exit 1; }
tail -1 $O/r50.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --model resnet50 --steps 8 --warmup 3 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$O/prof.log; exit 1; }
cd $GRAFT_REPO_ROOT
python3 scripts/copybuf_origin.py $(ls $O/prof/*kernel_trace.csv | head -1) stem_fwd --steps 3 > $O/copybuf.txt && cat $O/copybuf.txt
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE" \
           "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_sum" \
           "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $O/pmc_$i -o run -- python3 bench/write_roofline.py --reps 5 > $O/pmc_$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $O/pmc_$i.log; exit 1; }
done
python3 scripts/pmc_summary.py "$O/pmc_*/**/*counter_collection.csv" > $O/pmc_summary.csv
cat $O/pmc_summary.csv
