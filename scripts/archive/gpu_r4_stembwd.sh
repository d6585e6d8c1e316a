# ResNet-50 stem backward: max-pool backward fused into the BN backward (pool3_bn_bwd) vs maxpool3_bwd + bn_bwd_*,
# alternating on one box
set -o pipefail
O=gpurun_out/r4stembwd
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_norm_gpu.py tests/test_resnet.py -m gpu > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -30; exit $rc; }
for r in 1 2 3; do
  for v in 0 1; do
    AB_NOBWD=$v timeout -k 10 300 python3 bench.py --model resnet50 --steps 20 --warmup 5 > $O/r50_${v}_$r.log 2>&1 || { tail -5 $O/r50_${v}_$r.log; exit 1; }
    echo "nobwd=$v $(grep -o '"value": [0-9.]*' $O/r50_${v}_$r.log) $(grep -o '"ms_per_step": [0-9.]*' $O/r50_${v}_$r.log)"
  done
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --model resnet50 --steps 8 --warmup 5 --prewarm_ms 0 > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); python3 scripts/kstats.py "$f" > $O/r50_kernels.txt; grep -E "pool3|maxpool|stem" $O/r50_kernels.txt
