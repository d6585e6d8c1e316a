# LSTM staging kernel + kernel-gradient GEMM sweep + reference workloads (one GPU)
set -o pipefail
O=gpurun_out/r2j
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_models_gpu.py tests/test_kernels_gpu.py -k "lstm or seq_stage or small" > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -20; exit $rc; }
timeout -k 10 120 python3 bench/lstm_wgrad_sweep.py > $O/lstm_wgrad.txt 2>&1; cat $O/lstm_wgrad.txt
timeout -k 10 200 python3 bench/ref_models.py --steps 300 --warmup 30 > $O/ref_models.txt 2>&1 && grep '^{' $O/ref_models.txt
