# Round 5 A/B: one-replica CNN step with the fc/head Adam on a grid-capped side branch beside the
# conv backward (DTFE_CNN_FC_ADAM_SIDE=<workgroups>; 0 = the whole-model Adam after the join)
set -o pipefail
O=gpurun_out/${1:-r5fcside}
mkdir -p $O
DTFE_CNN_FC_ADAM_SIDE=32 timeout -k 10 300 python3 -u -m pytest tests/test_mnist_cnn_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -30; exit $rc; }
for rep in 1 2; do
for side in 0 16 32 64 128 0; do
for pw in 150 0; do
  DTFE_CNN_FC_ADAM_SIDE=$side timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --prewarm_ms $pw > $O/cnn_s${side}_pw$pw.log 2>&1 || { tail -5 $O/cnn_s${side}_pw$pw.log; exit 1; }
  echo "rep $rep side=$side prewarm=$pw $(grep -o '"ms_per_step": [0-9.]*' $O/cnn_s${side}_pw$pw.log)"
done; done; done
cd /tmp && export TMPDIR=/tmp
for side in 0 32; do
  DTFE_CNN_FC_ADAM_SIDE=$side timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_s$side -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 > $GRAFT_REPO_ROOT/$O/prof_s$side.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$O/prof_s$side.log; exit 1; }
done
echo done
