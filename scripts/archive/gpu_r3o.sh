# fc1 GEMM tile / split-K re-sweep (128x128 split-K halves the L2->LDS bytes of 64x64 tiles).
set -o pipefail
O=gpurun_out/r3o
mkdir -p $O
timeout -k 10 300 python3 bench/gemm_sweep.py --iters 20 --tiles 5,9,6,10,8,12 > $O/sweep.log 2>&1; cat $O/sweep.log
