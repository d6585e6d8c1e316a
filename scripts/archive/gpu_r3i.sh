# conv2 fixed kernels: pinned MFMA/read interleave + hoisted per-lane geometry + compile-time act;
# fc1 GEMM PMC (why ~13% MFMA busy); counter list for later passes.
set -o pipefail
O=gpurun_out/r3i
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_imgconv.py tests/test_mnist_cnn_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -20; exit $rc; }
timeout -k 10 120 python3 bench/cnn_kernels.py --iters 30 --only conv2_fwd,conv2_dgrad,conv2_wgrad,fc1_fwd,fc1_dgrad,fc1_wgrad > $O/k.log 2>&1; cat $O/k.log
for r in 1 2; do
  timeout -k 10 120 python3 bench.py > $O/b$r.log 2>&1 || exit 1; grep -o '"ms_per_step": [0-9.]*' $O/b$r.log
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -s KILL 60 rocprofv3 --list-avail > $O/avail.txt 2>&1
grep -o "^[A-Za-z0-9_]*TC[CP]_[A-Za-z0-9_]*\|^[A-Za-z0-9_]*TA_[A-Za-z0-9_]*" $O/avail.txt | head -0
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD" \
           "SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d $O/pmc_$i -o run -- python3 bench/cnn_kernels.py --iters 3 --only conv2_fwd,conv2_dgrad,fc1_fwd,fc1_dgrad,fc1_wgrad > $O/pmc_$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $O/pmc_$i.log; exit 1; }
  python3 scripts/pmc_summary.py "$O/pmc_$i/**/*counter_collection.csv" > $O/pmc_$i.csv; cat $O/pmc_$i.csv
done
exit 0
