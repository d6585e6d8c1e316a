# igemm weight-gradient split reduce with split slices per position (small weights x many splits fill
# the chip) vs the previous position-only reduce (A/B library): ResNet GPU tests + ResNet-50 step A/B.
set -o pipefail
O=gpurun_out/r3zf
mkdir -p $O
OLD=distributed-tensorflow-examples_amd/_C/ab/libdtfe_kernels.so
timeout -k 10 400 python3 -u -m pytest tests/test_resnet.py tests/test_igemm_gpu.py tests/test_igemm_tiles_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -1 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -20; exit $rc; }
for r in 1 2 3; do
  for v in new old; do
    if [ $v = old ]; then export DTFE_KERNEL_LIB=$OLD; else unset DTFE_KERNEL_LIB; fi
    timeout -k 10 300 python3 bench.py --model resnet50 --steps 20 --warmup 5 > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
    echo "$v $(grep -o '"value": [0-9.]*' $O/b.log) $(grep -o '"ms_per_step": [0-9.]*' $O/b.log)"
  done
done
unset DTFE_KERNEL_LIB
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --model resnet50 --steps 8 --warmup 5 > $O/prof.log 2>&1 || exit 1
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); python3 scripts/kstats.py "$f" > $O/r50_kernels.txt; grep -E "reduce|per-step" $O/r50_kernels.txt
exit 0
