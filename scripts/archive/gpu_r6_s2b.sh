# Round 6 (session 2): after removing the fused output statistics - imgconv / resnet GPU tests, ResNet-20 bench
set -o pipefail
O=gpurun_out/${1:-r6s2b}
mkdir -p $O
timeout -k 10 200 python3 bench.py --model resnet20 --steps 20 --warmup 5 > $O/r20.log 2>&1 || { tail -5 $O/r20.log; exit 1; }
echo "r20 $(grep -o '"ms_per_step": [0-9.]*' $O/r20.log)"
timeout -k 10 500 python3 -u -m pytest tests/test_imgconv.py tests/test_resnet.py -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -30; exit $rc; }
