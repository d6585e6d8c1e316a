# Round 5: weight-gradient grid target 512 px per workgroup for the k-group configs, same-box A/B vs HEAD
set -o pipefail
O=gpurun_out/r5wgpx
mkdir -p $O
AB=distributed-tensorflow-examples_amd/_C/ab/libdtfe_kernels.so
timeout -k 10 300 python3 -u -m pytest tests/test_imgconv.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -30; exit $rc; }
for v in new old; do
  if [ $v = old ]; then export DTFE_KERNEL_LIB=$AB; else unset DTFE_KERNEL_LIB; fi
  timeout -k 10 120 python3 bench/resnet20_kernels.py --only "wgrad" > $O/k_$v.txt 2>&1 || { tail -5 $O/k_$v.txt; exit 1; }
  echo "== $v"; grep -v amdgpu.ids $O/k_$v.txt
done
for rep in 1 2 3; do
for v in new old; do
  if [ $v = old ]; then export DTFE_KERNEL_LIB=$AB; else unset DTFE_KERNEL_LIB; fi
  timeout -k 10 200 python3 bench.py --model resnet20 --steps 20 --warmup 5 > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
  echo "$v $(grep -o '"ms_per_step": [0-9.]*' $O/b.log)"
done; done
