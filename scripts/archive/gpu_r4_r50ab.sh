# Round-4: ResNet-50 B=256 end to end with the persistent implicit GEMM off / only for the
# BN-backward-fused data gradients / everywhere (DTFE_PW), twice interleaved.
set -o pipefail
O=gpurun_out/r50ab
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_igemm_pw_gpu.py tests/test_resnet.py -m gpu > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -30; exit $rc; }
for r in 1 2; do
  for m in off bb all; do
    DTFE_PW=$m timeout -k 10 300 python3 bench.py --model resnet50 --steps 20 --warmup 5 > $O/r50_${m}_$r.log 2>&1 || { tail -5 $O/r50_${m}_$r.log; exit 1; }
    echo "$m $r $(grep -o '"value": [0-9.]*' $O/r50_${m}_$r.log) $(grep -o '"ms_per_step": [0-9.]*' $O/r50_${m}_$r.log)"
  done
done
