# BN statistics flush A/B (atomics after a tree LDS reduce vs workgroup slots + reduce launch)
set -o pipefail
O=gpurun_out/r2o
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_norm_gpu.py tests/test_resnet.py > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -20; exit $rc; }
for v in 0 1; do
DTFE_BN_SLOTS=$v timeout -k 10 240 python3 bench.py --model resnet20 --steps 50 --warmup 10 > $O/b_r20_$v.log 2>&1 && echo "slots=$v $(grep '^{' $O/b_r20_$v.log | cut -c1-170)" &&
DTFE_BN_SLOTS=$v timeout -k 10 300 python3 bench.py --model resnet50 --steps 20 --warmup 5 > $O/b_r50_$v.log 2>&1 && echo "slots=$v $(grep '^{' $O/b_r50_$v.log | cut -c1-170)" || exit 1
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_r20 -o run -- python3 bench.py --model resnet20 --steps 20 --warmup 5 > $O/prof_r20.log 2>&1 || exit 1
f=$(find $O/prof_r20 -name "*kernel_stats.csv" | head -1); python3 scripts/kstats.py "$f" > $O/r20_kernels.txt; head -14 $O/r20_kernels.txt
