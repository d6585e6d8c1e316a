# Write-through split-K slabs (fc1 forward split-K), head-less grouped fc launch, BN compile-time modes (A/B vs the
# previous norm.hip through DTFE_KERNEL_LIB).
set -o pipefail
O=gpurun_out/r3p
mkdir -p $O
OLD=distributed-tensorflow-examples_amd/_C/ab/libdtfe_kernels.so
timeout -k 10 400 python3 -u -m pytest tests/test_gemm_glds_gpu.py tests/test_kernels_gpu.py tests/test_norm_gpu.py tests/test_mnist_cnn_gpu.py tests/test_resnet.py -x -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -20; exit $rc; }
timeout -k 10 300 python3 bench/gemm_sweep.py --iters 20 --tiles 8,12 > $O/sweep.log 2>&1; cat $O/sweep.log
for r in 1 2; do
  for v in "0 1" "1 1" "0 2" "0 3" "1 3"; do
    set -- $v
    DTFE_CNN_FC_GROUP=$1 DTFE_CNN_FWD_SPLITS=$2 timeout -k 10 120 python3 bench.py > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
    echo "group=$1 fwd_splits=$2 $(grep -o '"ms_per_step": [0-9.]*' $O/b.log)"
  done
done
for r in 1 2; do
  for lib in new old; do
    if [ $lib = old ]; then export DTFE_KERNEL_LIB=$OLD; else unset DTFE_KERNEL_LIB; fi
    timeout -k 10 200 python3 bench.py --model resnet50 --steps 20 --warmup 5 > $O/r50.log 2>&1 || { tail -5 $O/r50.log; exit 1; }
    echo "resnet50 bn=$lib $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' $O/r50.log | tr '\n' ' ')"
  done
done
unset DTFE_KERNEL_LIB
timeout -k 10 200 python3 bench/bn_bench.py --batch 256 > $O/bn_new.txt 2>&1; cat $O/bn_new.txt
DTFE_KERNEL_LIB=$OLD timeout -k 10 200 python3 bench/bn_bench.py --batch 256 > $O/bn_old.txt 2>&1; cat $O/bn_old.txt
exit 0
