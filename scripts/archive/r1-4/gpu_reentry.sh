# Re-entry check on a fresh MI355X: GPU test suite, smoke(), default bench, ResNet-50 B=256 bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/gputests.log 2>&1 &&
timeout -k 10 180 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 180 python3 bench.py > gpurun_out/b_default.log 2>&1 &&
timeout -k 10 300 python3 bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/b_r50.log 2>&1
rc=$?
tail -n 3 gpurun_out/gputests.log; tail -n 1 gpurun_out/smoke.log; tail -n 1 gpurun_out/b_default.log; tail -n 1 gpurun_out/b_r50.log
exit $rc
