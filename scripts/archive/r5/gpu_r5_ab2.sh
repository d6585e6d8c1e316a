# Round 5 same-box A/B #2: register BN-statistics epilogue (HEAD) vs the round-4 LDS row-group epilogue
set -o pipefail
O=gpurun_out/${1:-r5ab2}
mkdir -p $O
AB=distributed-tensorflow-examples_amd/_C/ab/libdtfe_kernels.so
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_igemm_gpu.py tests/test_resnet.py > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -30; exit $rc; }
for r in 1 2; do
  for v in new old; do
    if [ $v = old ]; then export DTFE_KERNEL_LIB=$AB; else unset DTFE_KERNEL_LIB; fi
    timeout -k 10 200 python3 bench/write_roofline.py > $O/wr_${v}_$r.txt 2>&1 || { tail -5 $O/wr_${v}_$r.txt; exit 1; }
    echo "== $v $r"; grep conv $O/wr_${v}_$r.txt
    timeout -k 10 300 python3 bench.py --model resnet50 --steps 20 --warmup 5 > $O/r50_${v}_$r.log 2>&1 || { tail -5 $O/r50_${v}_$r.log; exit 1; }
    echo "r50 $v $r $(grep -o '"value": [0-9.]*' $O/r50_${v}_$r.log) $(grep -o '"ms_per_step": [0-9.]*' $O/r50_${v}_$r.log)"
  done
done
