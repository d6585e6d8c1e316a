# Round-2 final check on one GPU: the whole GPU suite, smoke(), default bench (driver contract), headline
# bench, ResNet-20/50, reference workloads, PS 1+2, CNN kernel stats + step timeline
set -o pipefail
O=gpurun_out/r2u
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -1 $O/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 180 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && tail -n 1 $O/smoke.log &&
timeout -k 10 180 python3 bench.py > $O/b_default.log 2>&1 && grep '^{' $O/b_default.log | cut -c1-200 &&
timeout -k 10 180 python3 bench.py --steps 300 --warmup 30 > $O/b_cnn.log 2>&1 && grep '^{' $O/b_cnn.log | cut -c1-200 &&
timeout -k 10 240 python3 bench.py --model resnet20 --steps 100 --warmup 10 > $O/b_r20.log 2>&1 && grep '^{' $O/b_r20.log | cut -c1-200 &&
timeout -k 10 300 python3 bench.py --model resnet50 --steps 20 --warmup 5 > $O/b_r50.log 2>&1 && grep '^{' $O/b_r50.log | cut -c1-200 &&
timeout -k 10 200 python3 bench/ref_models.py --steps 300 --warmup 30 > $O/ref_models.txt 2>&1 && grep '^{' $O/ref_models.txt &&
timeout -k 10 240 python3 bench.py --mode ps --gpus 2 --steps 50 --warmup 5 > $O/b_ps2.log 2>&1 && grep '^{' $O/b_ps2.log | cut -c1-200 || exit 1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_cnn -o run -- python3 bench.py --steps 30 --warmup 5 > $O/prof_cnn.log 2>&1 || exit 1
f=$(find $O/prof_cnn -name "*kernel_stats.csv" | head -1); python3 scripts/kstats.py "$f" > $O/cnn_kernels.txt
f=$(find $O/prof_cnn -name "*kernel_trace.csv" | head -1); python3 scripts/timeline.py "$f" conv1c_fwd > $O/cnn_timeline.txt; cat $O/cnn_timeline.txt
