# fused head weight gradient in the fc1 dgrad launch: kernel + CNN tests (incl. 2-rank IPC in-graph), A/B bench, timeline
set -o pipefail
O=gpurun_out/r2q
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_mnist_cnn_gpu.py > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -20; exit $rc; }
b() { tag=$(echo "$*" | tr ' =' '_-'); timeout -k 10 180 env "$@" python3 bench.py --steps 300 --warmup 30 > $O/b_$tag.log 2>&1 && echo "$* $(grep '^{' $O/b_$tag.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["median_window_ms_per_step"])')"; }
b DTFE_CNN_HEAD_FUSE=1 DTFE_CNN_FC1W_SPLIT=2 && b DTFE_CNN_HEAD_FUSE=0 && b DTFE_CNN_HEAD_FUSE=1 DTFE_CNN_FC1W_SPLIT=2 && b DTFE_CNN_HEAD_FUSE=0 && b DTFE_CNN_HEAD_FUSE=0 DTFE_CNN_FC1W_SPLIT=2 || exit 1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
DTFE_CNN_HEAD_FUSE=1 DTFE_CNN_FC1W_SPLIT=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_cnn -o run -- python3 bench.py --steps 30 --warmup 5 > $O/prof_cnn.log 2>&1 || exit 1
f=$(find $O/prof_cnn -name "*kernel_stats.csv" | head -1); python3 scripts/kstats.py "$f" > $O/cnn_kernels.txt
f=$(find $O/prof_cnn -name "*kernel_trace.csv" | head -1); python3 scripts/timeline.py "$f" conv1c_fwd > $O/cnn_timeline.txt; cat $O/cnn_timeline.txt
