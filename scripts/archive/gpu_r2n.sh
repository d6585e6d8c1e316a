# BN statistics without same-address atomics: BN/ResNet tests, ResNet-20 / ResNet-50 benches, R20 kernel stats
set -o pipefail
O=gpurun_out/r2n
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_norm_gpu.py tests/test_resnet.py tests/test_stem_gpu.py > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -20; exit $rc; }
timeout -k 10 240 python3 bench.py --model resnet20 --steps 50 --warmup 10 > $O/b_r20.log 2>&1 && grep '^{' $O/b_r20.log | cut -c1-250 &&
timeout -k 10 300 python3 bench.py --model resnet50 --steps 20 --warmup 5 > $O/b_r50.log 2>&1 && grep '^{' $O/b_r50.log | cut -c1-250 || exit 1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_r20 -o run -- python3 bench.py --model resnet20 --steps 20 --warmup 5 > $O/prof_r20.log 2>&1 || exit 1
f=$(find $O/prof_r20 -name "*kernel_stats.csv" | head -1); python3 scripts/kstats.py "$f" > $O/r20_kernels.txt; head -30 $O/r20_kernels.txt
