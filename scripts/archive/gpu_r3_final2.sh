# Round-3 closing check #2 (after the head-in-group and split-reduce changes): ResNet weight-gradient
# split-reduce A/B vs the previous reduce (A/B library), then the full GPU suite, smoke(), the bench
# lines and the MNIST CNN timeline / kernel table.
set -o pipefail
O=gpurun_out/r3final2
mkdir -p $O
OLD=distributed-tensorflow-examples_amd/_C/ab/libdtfe_kernels.so
for r in 1 2 3; do
  for v in new old; do
    if [ $v = old ]; then export DTFE_KERNEL_LIB=$OLD; else unset DTFE_KERNEL_LIB; fi
    timeout -k 10 300 python3 bench.py --model resnet50 --steps 20 --warmup 5 > $O/b_ab.log 2>&1 || { tail -5 $O/b_ab.log; exit 1; }
    echo "reduce=$v $(grep -o '"value": [0-9.]*' $O/b_ab.log) $(grep -o '"ms_per_step": [0-9.]*' $O/b_ab.log)"
  done
done
unset DTFE_KERNEL_LIB
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $O/gputests.log 2>&1 &&
timeout -k 10 180 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 180 python3 bench.py > $O/b_default.log 2>&1 &&
timeout -k 10 180 python3 bench.py --steps 20 --warmup 5 > $O/b_driver.log 2>&1 &&
timeout -k 10 300 python3 bench.py --model resnet20 --steps 20 --warmup 5 > $O/b_r20.log 2>&1 &&
timeout -k 10 300 python3 bench.py --model resnet50 --steps 20 --warmup 5 > $O/b_r50.log 2>&1
rc=$?
tail -n 1 $O/gputests.log; tail -n 1 $O/smoke.log; tail -n 1 $O/b_default.log; tail -n 1 $O/b_driver.log; tail -n 1 $O/b_r20.log; tail -n 1 $O/b_r50.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/gputests.log | head -10; exit $rc; }
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_cnn -o run -- python3 bench.py --steps 30 --warmup 5 > $O/prof_cnn.log 2>&1 || exit 1
f=$(find $O/prof_cnn -name "*kernel_stats.csv" | head -1); python3 scripts/kstats.py "$f" > $O/cnn_kernels.txt; head -16 $O/cnn_kernels.txt
f=$(find $O/prof_cnn -name "*kernel_trace.csv" | head -1); python3 scripts/timeline.py "$f" conv1c_fwd > $O/cnn_timeline.txt; cat $O/cnn_timeline.txt
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_r50 -o run -- python3 bench.py --model resnet50 --steps 8 --warmup 5 > $O/prof_r50.log 2>&1 || exit 1
f=$(find $O/prof_r50 -name "*kernel_stats.csv" | head -1); python3 scripts/kstats.py "$f" > $O/r50_kernels.txt; head -24 $O/r50_kernels.txt
exit 0
