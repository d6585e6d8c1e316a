set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -m pytest tests/test_igemm_gpu.py -x -q > gpurun_out/pytest_igemm.log 2>&1 &&
timeout -k 10 300 python3 bench/resnet50_convs.py > gpurun_out/r50_convs.log 2>&1 &&
timeout -k 10 300 python3 bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/b_r50.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_igemm.log; cat gpurun_out/r50_convs.log; cat gpurun_out/b_r50.log
exit $rc
