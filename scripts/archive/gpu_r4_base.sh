# Round-4 baseline on a fresh box: GPU suite, smoke, driver-shaped CNN bench, ResNet-50 bench and
# the per-layer ResNet-50 conv table (B=256).
set -o pipefail
O=gpurun_out/r4base
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $O/gputests.log 2>&1 &&
timeout -k 10 180 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 180 python3 bench.py --steps 20 --warmup 5 > $O/b_driver.log 2>&1 &&
timeout -k 10 300 python3 bench.py --model resnet50 --steps 20 --warmup 5 > $O/b_r50.log 2>&1 &&
timeout -k 10 400 python3 bench/resnet50_convs.py --batch 256 --reps 10 --no-torch > $O/convs.txt 2>&1
rc=$?
tail -n 1 $O/gputests.log; tail -n 1 $O/smoke.log; tail -n 1 $O/b_driver.log; tail -n 1 $O/b_r50.log; tail -n 3 $O/convs.txt
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/gputests.log | head -10; exit $rc; }
exit 0
