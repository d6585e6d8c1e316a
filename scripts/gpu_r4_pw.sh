# Round-4: CNN schedule/fp32/evaluate tests, pointwise 1x1 GEMM tests, ResNet-50 conv table per DTFE_PW_CFG,
# ResNet-50 + CNN bench.
set -o pipefail
O=gpurun_out/r4pw
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_igemm_pw_gpu.py tests/test_igemm_gpu.py > $O/pytest_pw.log 2>&1
rc=$?; tail -3 $O/pytest_pw.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest_pw.log | head -30; exit $rc; }
for c in 0 1 2 3; do
  DTFE_PW_CFG=$c timeout -k 10 300 python3 bench/resnet50_convs.py --batch 256 --reps 10 --no-torch > $O/convs_cfg$c.txt 2>&1 || exit 1
  echo "cfg=$c $(tail -1 $O/convs_cfg$c.txt)"
done
DTFE_PW_OFF=1 timeout -k 10 300 python3 bench/resnet50_convs.py --batch 256 --reps 10 --no-torch > $O/convs_off.txt 2>&1 || exit 1
echo "off $(tail -1 $O/convs_off.txt)"
timeout -k 10 300 python3 bench.py --model resnet50 --steps 20 --warmup 5 > $O/b_r50.log 2>&1 && tail -1 $O/b_r50.log | cut -c1-150
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_mnist_cnn_gpu.py tests/test_rccl_gpu.py tests/test_cluster_gpu.py tests/test_kernels_gpu.py \
  -k "cnn or splitk" > $O/pytest_cnn.log 2>&1
rc=$?; tail -3 $O/pytest_cnn.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest_cnn.log | head -30; exit $rc; }
timeout -k 10 180 python3 bench.py --steps 20 --warmup 5 > $O/b_driver.log 2>&1 && tail -1 $O/b_driver.log | cut -c1-200
