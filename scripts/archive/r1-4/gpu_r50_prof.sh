# ResNet-50 B=256: resnet tests, bench, rocprofv3 kernel stats
set -o pipefail
O=gpurun_out/${1:-r2o}
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_resnet.py tests/test_stem_gpu.py tests/test_norm_gpu.py > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --model resnet50 --steps 20 --warmup 5 > $O/bench.log 2>&1 && grep '^{' $O/bench.log | cut -c1-240 || exit 1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --model resnet50 --steps 8 --warmup 5 > $O/prof.log 2>&1 || exit 1
f=$(find $O/prof -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && python3 scripts/kstats.py "$f" > $O/kernels.txt && head -40 $O/kernels.txt
exit 0
