set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -m pytest tests/test_imgconv.py -x -q > gpurun_out/t_img.log 2>&1; echo "TEST EXIT $?" >> gpurun_out/t_img.log
tail -3 gpurun_out/t_img.log
grep -q "TEST EXIT 0" gpurun_out/t_img.log || { grep -E "assert|Error" gpurun_out/t_img.log | head -20; exit 1; }
timeout -k 10 300 python3 bench/cnn_kernels.py --batch_size 1024 --iters 30 > gpurun_out/ck.log 2>&1 && cat gpurun_out/ck.log
timeout -k 10 300 python3 bench.py --steps 100 --warmup 10 > gpurun_out/bench.log 2>&1; tail -2 gpurun_out/bench.log
