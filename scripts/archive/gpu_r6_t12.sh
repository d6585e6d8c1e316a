# Round 6: fused statistics with a DPP reduction: ablation, tests, ResNet-20 bench
set -o pipefail
O=gpurun_out/${1:-r6t12}
mkdir -p $O
for d in "" "icr=256" "icr=512"; do
  DTFE_DIAG=$d timeout -k 10 120 python3 bench/imgconv_stats_ab.py > $O/ab_$d.log 2>&1 || { tail -5 $O/ab_$d.log; exit 1; }
  grep -v amdgpu.ids $O/ab_$d.log
done
timeout -k 10 300 python3 -u -m pytest tests/test_imgconv.py tests/test_resnet.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -30; exit $rc; }
timeout -k 10 200 python3 bench.py --model resnet20 --steps 30 --warmup 10 > $O/r20.log 2>&1 || { tail -5 $O/r20.log; exit 1; }
tail -1 $O/r20.log | cut -c1-300
