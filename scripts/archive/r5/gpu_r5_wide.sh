# Round 5: register BN-statistics epilogue + 64x256 tile for one-k-tile 1x1 convs: tests, write roofline,
# ResNet-50 bench, kernel table
set -o pipefail
O=gpurun_out/${1:-r5wide}
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_igemm_gpu.py tests/test_resnet.py tests/test_norm_gpu.py tests/test_stem_gpu.py > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -30; exit $rc; }
timeout -k 10 200 python3 bench/write_roofline.py > $O/write_roofline.txt 2>&1 || { tail -5 $O/write_roofline.txt; exit 1; }
cat $O/write_roofline.txt | grep -v amdgpu
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --model resnet50 --steps 20 --warmup 5 > $O/r50_$r.log 2>&1 || { tail -5 $O/r50_$r.log; exit 1; }
  echo "r50 $r $(grep -o '"value": [0-9.]*' $O/r50_$r.log) $(grep -o '"ms_per_step": [0-9.]*' $O/r50_$r.log)"
done
timeout -k 10 300 python3 bench/resnet50_convs.py --batch 256 --reps 10 --no-torch > $O/convs.txt 2>&1 || { tail -5 $O/convs.txt; exit 1; }
tail -25 $O/convs.txt
