set -o pipefail
O=gpurun_out/r2c
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gemm_glds_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest_glds.log 2>&1
rc=$?; tail -15 $O/pytest_glds.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench/gemm_sweep.py --iters 20 > $O/gemm_sweep.txt 2>&1; cat $O/gemm_sweep.txt
DTFE_GLDS_STAGES=2 timeout -k 10 400 python3 bench/gemm_sweep.py --iters 20 > $O/gemm_sweep_s2.txt 2>&1; grep "x.*g " $O/gemm_sweep_s2.txt
