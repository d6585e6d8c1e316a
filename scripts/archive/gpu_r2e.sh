# Round-2 re-entry check on one GPU: the whole GPU suite, smoke(), the headline bench, ResNet-50
# at B=256, the reference workloads and the 1 ps + 2 worker PS bench.  Each step has its own
# time limit; the chain stops at the first failure.
set -o pipefail
O=gpurun_out/r2e
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 180 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && tail -n 1 $O/smoke.log &&
timeout -k 10 180 python3 bench.py > $O/b_default.log 2>&1 && grep '^{' $O/b_default.log | cut -c1-260 &&
timeout -k 10 180 python3 bench.py --steps 200 --warmup 20 > $O/b_cnn.log 2>&1 && grep '^{' $O/b_cnn.log | cut -c1-260 &&
timeout -k 10 300 python3 bench.py --model resnet50 --steps 20 --warmup 5 > $O/b_r50.log 2>&1 && grep '^{' $O/b_r50.log | cut -c1-260 &&
timeout -k 10 200 python3 bench/ref_models.py --steps 300 --warmup 30 > $O/ref_models.txt 2>&1 && cat $O/ref_models.txt | tail -4 &&
timeout -k 10 240 python3 bench.py --mode ps --gpus 2 --steps 50 --warmup 5 > $O/b_ps2.log 2>&1 && grep '^{' $O/b_ps2.log | cut -c1-260
