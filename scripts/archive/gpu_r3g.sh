# Round-3 session 3: re-entry GPU check + conv2 backward attribution (isolated timings with diag variants, PMC).
set -o pipefail
O=gpurun_out/r3g
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $O/gputests.log 2>&1 &&
timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 > $O/b_driver.log 2>&1 &&
timeout -k 10 120 python3 bench.py > $O/b_default.log 2>&1 &&
timeout -k 10 120 python3 bench/cnn_kernels.py --iters 30 > $O/cnn_kernels.log 2>&1 &&
for d in 1 2 4 6 7; do
  DTFE_IC_DIAG=$d DTFE_IW_DIAG=$d timeout -k 10 60 python3 bench/cnn_kernels.py --iters 30 --only conv2_fwd,conv2_dgrad,conv2_wgrad > $O/cnn_diag$d.log 2>&1 || exit 1
done
rc=$?
tail -n 2 $O/gputests.log; tail -n 1 $O/b_driver.log; tail -n 1 $O/b_default.log; cat $O/cnn_kernels.log
for d in 1 2 4 6 7; do echo "diag $d"; cat $O/cnn_diag$d.log; done
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAVE_CYCLES" \
           "SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU"; do
  for d in 0 4; do
    i=$((i+1))
    DTFE_IC_DIAG=$d DTFE_IW_DIAG=$d timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d $O/pmc_$i -o run -- python3 bench/cnn_kernels.py --iters 3 --only conv2_fwd,conv2_dgrad,conv2_wgrad > $O/pmc_$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $O/pmc_$i.log; exit 1; }
    python3 scripts/pmc_summary.py "$O/pmc_$i/**/*counter_collection.csv" > $O/pmc_${i}_d$d.csv
  done
done
for f in $O/pmc_*_d*.csv; do echo "== $f"; cat $f; done
timeout -k 10 400 python3 bench/resnet50_convs.py --batch 256 --reps 10 > $O/r50_convs.log 2>&1; cat $O/r50_convs.log
exit 0
