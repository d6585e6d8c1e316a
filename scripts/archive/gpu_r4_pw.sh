# Round-4: pipelined implicit-GEMM kernels (fwd/dgrad one-phase launches + BN statistics epilogues, pipelined
# wgrad), ResNet-50 conv table per configuration vs the round-3 kernels, ResNet-50 bench, CNN / comm tests.
set -o pipefail
O=gpurun_out/r4pw
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_igemm_pw_gpu.py tests/test_igemm_gpu.py tests/test_resnet.py -k "not stock_amp" > $O/pytest_pw.log 2>&1
rc=$?; tail -3 $O/pytest_pw.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest_pw.log | head -30; exit $rc; }
run_tab() {  # name, env...
  n=$1; shift
  env "$@" timeout -k 10 300 python3 bench/resnet50_convs.py --batch 256 --reps 10 --no-torch > $O/convs_$n.txt 2>&1 || exit 1
  echo "$n $(tail -1 $O/convs_$n.txt)"
}
run_tab new DTFE_IG_WPIPE=1
run_tab cfg1_w2 DTFE_PW_CFG=1 DTFE_IG_WPIPE=2
run_tab cfg2_w0 DTFE_PW_CFG=2 DTFE_IG_WPIPE=0
run_tab old DTFE_PW_OFF=1 DTFE_IG_WPIPE=0
for v in 0 1; do
  DTFE_PW_OFF=$v timeout -k 10 300 python3 bench.py --model resnet50 --steps 20 --warmup 5 > $O/b_r50_off$v.log 2>&1 || exit 1
  echo "pw_off=$v $(tail -1 $O/b_r50_off$v.log | cut -c1-140)"
done
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_mnist_cnn_gpu.py tests/test_rccl_gpu.py tests/test_cluster_gpu.py tests/test_kernels_gpu.py \
  -k "cnn or splitk or crash" > $O/pytest_cnn.log 2>&1
rc=$?; tail -3 $O/pytest_cnn.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest_cnn.log | head -30; exit $rc; }
for r in 1 2; do for v in 0 1; do
  DTFE_CNN_FC_ADAM_SIDE=$v timeout -k 10 180 python3 bench.py --steps 200 --warmup 20 > $O/b_fcside$v.log 2>&1 || exit 1
  echo "fc_adam_side=$v $(grep -o '"ms_per_step": [0-9.]*' $O/b_fcside$v.log) $(grep -o '"median_window_ms_per_step": [0-9.]*' $O/b_fcside$v.log)"
done; done
