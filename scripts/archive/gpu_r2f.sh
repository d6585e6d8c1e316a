# Round-2 session-4 check: the whole GPU suite,
# smoke, benches and the reference workloads.  Each GPU step has its own time limit.
set -o pipefail
O=gpurun_out/r2f
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 180 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && tail -n 1 $O/smoke.log &&
timeout -k 10 180 python3 bench.py --steps 200 --warmup 20 > $O/b_cnn.log 2>&1 && grep '^{' $O/b_cnn.log | cut -c1-330 &&
timeout -k 10 300 python3 bench.py --model resnet50 --steps 20 --warmup 5 > $O/b_r50.log 2>&1 && grep '^{' $O/b_r50.log | cut -c1-260 &&
timeout -k 10 200 python3 bench/ref_models.py --steps 300 --warmup 30 > $O/ref_models.txt 2>&1 && tail -4 $O/ref_models.txt &&
timeout -k 10 240 python3 bench.py --mode ps --gpus 2 --steps 50 --warmup 5 > $O/b_ps2.log 2>&1 && grep '^{' $O/b_ps2.log | cut -c1-260
