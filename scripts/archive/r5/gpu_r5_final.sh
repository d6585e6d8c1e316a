# Round 5 final check: every GPU test, smoke(), the driver-shaped benches (CNN with/without pre-warm,
# ResNet-20, ResNet-50), and a ResNet-20 kernel trace (per-kernel table + launch count)
set -o pipefail
O=gpurun_out/${1:-r5final}
mkdir -p $O
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -30; exit $rc; }
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && tail -1 $O/smoke.log || { tail -5 $O/smoke.log; exit 1; }
for pw in 150 0; do
  timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --prewarm_ms $pw > $O/cnn_pw$pw.log 2>&1 || { tail -5 $O/cnn_pw$pw.log; exit 1; }
  echo "cnn prewarm=$pw $(grep -o '"value": [0-9.]*' $O/cnn_pw$pw.log) $(grep -o '"ms_per_step": [0-9.]*' $O/cnn_pw$pw.log)"
done
for m in resnet20 resnet50; do
  timeout -k 10 300 python3 bench.py --model $m --steps 20 --warmup 5 > $O/$m.log 2>&1 || { tail -5 $O/$m.log; exit 1; }
  echo "$m $(grep -o '"value": [0-9.]*' $O/$m.log) $(grep -o '"ms_per_step": [0-9.]*' $O/$m.log)"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/r20prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --model resnet20 --steps 20 --warmup 5 > $GRAFT_REPO_ROOT/$O/r20prof.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$O/r20prof.log; exit 1; }
echo done
