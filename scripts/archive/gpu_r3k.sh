# fc1 GEMM memory-path PMC: TLB (UTCL1) hit/miss, L2 read latency, TA/TCP stalls.
set -o pipefail
O=${O:-gpurun_out/r3k}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
i=0
for set in "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE" \
           "TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_ADDR_STALL_CYCLES_sum TCP_UTCL1_STALL_MULTI_MISS_sum TCP_TCR_TCP_STALL_CYCLES_sum TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE" \
           "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_LEVEL_sum TCC_BUSY_sum TCC_TAG_STALL_sum GRBM_GUI_ACTIVE SQ_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d $O/pmc_$i -o run -- python3 bench/cnn_kernels.py --iters 3 --only fc1_fwd,fc1_dgrad,fc1_wgrad,conv2_fwd > $O/pmc_$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $O/pmc_$i.log; continue; }
  python3 scripts/pmc_summary.py "$O/pmc_$i/**/*counter_collection.csv" > $O/pmc_$i.csv; cat $O/pmc_$i.csv
done
exit 0
