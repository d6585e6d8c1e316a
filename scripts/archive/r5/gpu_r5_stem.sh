# Round 5: vectorized few-channel image staging (ResNet-20 stem fwd / wgrad, small-batch MNIST conv1):
# numerics, then a same-box A/B against the HEAD library
set -o pipefail
O=gpurun_out/r5stem
mkdir -p $O
AB=distributed-tensorflow-examples_amd/_C/ab/libdtfe_kernels.so
timeout -k 10 400 python3 -u -m pytest tests/test_imgconv.py tests/test_resnet.py tests/test_kernels_gpu.py tests/test_mnist_cnn_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -30; exit $rc; }
for rep in 1 2 3; do
for v in new old; do
  if [ $v = old ]; then export DTFE_KERNEL_LIB=$AB; else unset DTFE_KERNEL_LIB; fi
  timeout -k 10 200 python3 bench.py --model resnet20 --steps 20 --warmup 5 > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
  echo "$v $(grep -o '"ms_per_step": [0-9.]*' $O/b.log)"
done; done
unset DTFE_KERNEL_LIB
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --model resnet20 --steps 10 --warmup 3 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$O/prof.log; exit 1; }
echo done
