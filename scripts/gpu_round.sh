set -o pipefail
mkdir -p gpurun_out
python3 -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 &&
timeout -k 10 900 python3 -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 200 python3 bench.py --steps 200 --warmup 20 > gpurun_out/b_cnn.log 2>&1 &&
timeout -k 10 200 python3 bench.py --model resnet20 --steps 50 --warmup 10 > gpurun_out/b_r20.log 2>&1 &&
timeout -k 10 300 python3 bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/b_r50.log 2>&1 &&
timeout -k 10 300 python3 bench/stock_torch_resnet.py --arch resnet20 --steps 50 --warmup 10 > gpurun_out/s_r20.log 2>&1 &&
timeout -k 10 400 python3 bench/stock_torch_resnet.py --arch resnet50 --steps 20 --warmup 5 > gpurun_out/s_r50.log 2>&1
rc=$?
tail -2 gpurun_out/pytest_gpu.log; for f in gpurun_out/b_*.log gpurun_out/s_*.log; do tail -n 1 $f; done
exit $rc
