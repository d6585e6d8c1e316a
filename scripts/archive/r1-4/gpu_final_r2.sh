# Round-2 closing check on a fresh MI355X: full GPU suite, smoke(), default bench (driver contract),
# ResNet-50 B=256 bench, and rocprofv3 kernel stats of the ResNet-50 and MNIST CNN steps.
set -o pipefail
O=gpurun_out/final
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $O/gputests.log 2>&1 &&
timeout -k 10 180 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 180 python3 bench.py > $O/b_default.log 2>&1 &&
timeout -k 10 300 python3 bench.py --model resnet50 --steps 20 --warmup 5 > $O/b_r50.log 2>&1 &&
timeout -k 10 200 python3 bench.py --model resnet20 > $O/b_r20.log 2>&1
rc=$?
tail -n 2 $O/gputests.log; tail -n 1 $O/smoke.log; tail -n 1 $O/b_default.log; tail -n 1 $O/b_r50.log; tail -n 1 $O/b_r20.log
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_r50 -o run -- python3 bench.py --model resnet50 --steps 8 --warmup 5 > $O/prof_r50.log 2>&1 || exit 1
f=$(find $O/prof_r50 -name "*kernel_stats.csv" | head -1); python3 scripts/kstats.py "$f" > $O/r50_kernels.txt; head -30 $O/r50_kernels.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_cnn -o run -- python3 bench.py --steps 30 --warmup 5 > $O/prof_cnn.log 2>&1 || exit 1
f=$(find $O/prof_cnn -name "*kernel_stats.csv" | head -1); python3 scripts/kstats.py "$f" > $O/cnn_kernels.txt; head -20 $O/cnn_kernels.txt
exit 0
