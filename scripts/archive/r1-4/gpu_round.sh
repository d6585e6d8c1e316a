# One GPU call: kernel/model tests, headline + ResNet benches, rocprof stats.
# The .so files are built in-tree on the CPU host beforehand (they travel with the snapshot).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 200 python3 bench.py --steps 200 --warmup 20 > gpurun_out/b_cnn.log 2>&1 &&
timeout -k 10 200 python3 bench.py --model resnet20 --steps 50 --warmup 10 > gpurun_out/b_r20.log 2>&1 &&
timeout -k 10 300 python3 bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/b_r50.log 2>&1 &&
bash scripts/profile.sh r50 --model resnet50 --steps 10 --warmup 3 > gpurun_out/prof_r50.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu.log; for f in gpurun_out/b_*.log; do tail -n 1 $f; done
exit $rc
