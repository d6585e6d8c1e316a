# Round-2 profiling pass on one GPU: CNN schedule A/B (env switches), CNN step timeline,
# ResNet-50 B=256 kernel stats, LSTM/GAN traces.  Each GPU step has its own time limit.
set -o pipefail
O=gpurun_out/r2g
mkdir -p $O
b() { timeout -k 10 180 env "$@" python3 bench.py --steps 300 --warmup 30 > $O/b_$1.log 2>&1 && echo "$1 $(grep '^{' $O/b_$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["median_window_ms_per_step"])')"; }
b DTFE_X=base && b DTFE_CNN_EARLY_APPLY=1 && b DTFE_CNN_HEAD_GEMM=1 && b DTFE_CNN_BRANCHES=side1 && b DTFE_CNN_ORDER=crit || exit 1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_cnn -o run -- python3 bench.py --steps 30 --warmup 5 > $O/prof_cnn.log 2>&1 || exit 1
f=$(find $O/prof_cnn -name "*kernel_stats.csv" | head -1); python3 scripts/kstats.py "$f" > $O/cnn_kernels.txt
f=$(find $O/prof_cnn -name "*kernel_trace.csv" | head -1); python3 scripts/timeline.py "$f" conv1c_fwd > $O/cnn_timeline.txt; cat $O/cnn_timeline.txt
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_r50 -o run -- python3 bench.py --model resnet50 --steps 8 --warmup 5 > $O/prof_r50.log 2>&1 || exit 1
f=$(find $O/prof_r50 -name "*kernel_stats.csv" | head -1); python3 scripts/kstats.py "$f" > $O/r50_kernels.txt; head -30 $O/r50_kernels.txt
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_lstm -o run -- python3 bench/ref_models.py --models lstm --steps 100 --warmup 10 > $O/prof_lstm.log 2>&1 || exit 1
f=$(find $O/prof_lstm -name "*kernel_stats.csv" | head -1); python3 scripts/kstats.py "$f" > $O/lstm_kernels.txt; cat $O/lstm_kernels.txt
f=$(find $O/prof_lstm -name "*kernel_trace.csv" | head -1); python3 scripts/trace_summary.py "$f" lstm > $O/lstm_trace.txt 2>&1; cat $O/lstm_trace.txt
exit 0
