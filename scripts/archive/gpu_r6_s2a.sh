# Round 6 (session 2): ResNet-20 fused output statistics as compile-time instances - isolated convs,
# step A/B (fused vs bn_stats pass), imgconv / resnet GPU tests
set -o pipefail
O=gpurun_out/${1:-r6s2a}
mkdir -p $O
timeout -k 10 120 python3 bench/imgconv_stats_ab.py > $O/ab.log 2>&1 || { tail -5 $O/ab.log; exit 1; }
grep -v amdgpu.ids $O/ab.log
timeout -k 10 300 python3 bench/r20_ostats_ab.py --rounds 2 > $O/r20ab.log 2>&1 || { tail -5 $O/r20ab.log; exit 1; }
grep out_stats $O/r20ab.log
timeout -k 10 400 python3 -u -m pytest tests/test_imgconv.py tests/test_resnet.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -30; exit $rc; }
