# Round-4: 32-deep k-tile 4-stage implicit GEMM (DTFE_IG_KB=32) - tests, conv tables, ResNet-50 A/B
set -o pipefail
O=gpurun_out/r4kb
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_igemm_gpu.py tests/test_igemm_tiles_gpu.py > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -30; exit $rc; }
for kb in 64 32; do
  DTFE_IG_KB=$kb timeout -k 10 300 python3 bench/resnet50_convs.py --batch 256 --reps 10 --no-torch > $O/convs_$kb.txt 2>&1 || exit 1
  echo "kb=$kb $(tail -1 $O/convs_$kb.txt)"
done
for r in 1 2; do
  for kb in 64 32; do
    DTFE_IG_KB=$kb timeout -k 10 300 python3 bench.py --model resnet50 --steps 20 --warmup 5 > $O/r50_${kb}_$r.log 2>&1 || { tail -5 $O/r50_${kb}_$r.log; exit 1; }
    echo "r50 kb=$kb $(grep -o '"value": [0-9.]*' $O/r50_${kb}_$r.log) $(grep -o '"ms_per_step": [0-9.]*' $O/r50_${kb}_$r.log)"
  done
done
