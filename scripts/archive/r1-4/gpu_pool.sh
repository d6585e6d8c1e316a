# max-pool backward (2x2-cell threads): norm/ResNet GPU tests, ResNet-50 bench, kernel stats.
set -o pipefail
O=gpurun_out/pool
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_norm_gpu.py tests/test_resnet.py -m gpu -x -q --timeout 120 \
  --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 &&
timeout -k 10 300 python3 bench.py --model resnet50 --steps 20 --warmup 5 > $O/b_r50.log 2>&1
rc=$?
tail -n 2 $O/tests.log; tail -n 1 $O/b_r50.log | cut -c1-400
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --model resnet50 --steps 8 --warmup 5 > $O/prof.log 2>&1 || exit 1
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); python3 scripts/kstats.py "$f" > $O/r50_kernels.txt; grep -E "maxpool|igemm_kernel|bn_" $O/r50_kernels.txt
exit 0
