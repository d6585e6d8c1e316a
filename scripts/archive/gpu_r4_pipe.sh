# Round-4: inline-asm DMA pipelines (wgrad ring, persistent fwd/dgrad) - tests, conv table per variant,
# PMC of one 3x3 and one 1x1 layer old vs persistent.
set -o pipefail
O=gpurun_out/r4pipe
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_igemm_pw_gpu.py tests/test_igemm_gpu.py > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -30; exit $rc; }
run_tab() {
  n=$1; shift
  env "$@" timeout -k 10 300 python3 bench/resnet50_convs.py --batch 256 --reps 10 --no-torch > $O/convs_$n.txt 2>&1 || exit 1
  echo "$n $(tail -1 $O/convs_$n.txt)"
}
run_tab old DTFE_PW=off DTFE_IG_WPIPE=0
#run_tab w1 DTFE_PW=off DTFE_IG_WPIPE=1
#run_tab w2 DTFE_PW=off DTFE_IG_WPIPE=2
run_tab pw0 DTFE_PW=all,cfg=0 DTFE_IG_WPIPE=0
run_tab pw1 DTFE_PW=all,cfg=1 DTFE_IG_WPIPE=0
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for v in off all; do
  DTFE_PW=$v,mintiles=1 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
    --output-format csv -d $O/pmc_$v -o run -- python3 bench/resnet50_convs.py --batch 256 --reps 3 --no-torch --only "14,256,256,3,1;14,1024,256,1,1" > $O/pmc_$v.log 2>&1 || { tail -5 $O/pmc_$v.log; exit 1; }
done
python3 scripts/pmc_summary.py "$O/pmc_*/**/*counter_collection.csv" > $O/pmc_summary.csv 2>&1; head -40 $O/pmc_summary.csv
