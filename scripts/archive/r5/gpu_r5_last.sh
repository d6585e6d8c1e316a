# Round 5 closing sanity on the committed tree: GPU tests, smoke, CNN and ResNet-20 benches
set -o pipefail
O=gpurun_out/r5last
mkdir -p $O
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -30; exit $rc; }
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && tail -1 $O/smoke.log || { tail -5 $O/smoke.log; exit 1; }
timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 > $O/cnn.log 2>&1 || { tail -5 $O/cnn.log; exit 1; }
tail -1 $O/cnn.log
timeout -k 10 200 python3 bench.py --model resnet20 --steps 20 --warmup 5 > $O/r20.log 2>&1 || { tail -5 $O/r20.log; exit 1; }
tail -1 $O/r20.log
