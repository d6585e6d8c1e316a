# conv1 weight-gradient kernel: grid sweep + ablation (bench step time; the kernel is on the step's tail)
set -o pipefail
O=gpurun_out/r2k
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_mnist_cnn_gpu.py tests/test_imgconv.py > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -20; exit $rc; }
b() { tag=$(echo "$*" | tr ' =' '_-'); timeout -k 10 180 env "$@" python3 bench.py --steps 300 --warmup 30 > $O/b_$tag.log 2>&1 && echo "$* $(grep '^{' $O/b_$tag.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["median_window_ms_per_step"])')"; }
b DTFE_C1W_GRID=256 && b DTFE_C1W_GRID=512 && b DTFE_C1W_GRID=1024 && b DTFE_C1W_GRID=128 && \
b DTFE_C1W_DIAG=1 && b DTFE_C1W_DIAG=2 && b DTFE_C1W_DIAG=4 && b DTFE_C1W_DIAG=8 && b DTFE_C1W_DIAG=15 || exit 1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
DTFE_C1W_GRID=512 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof512 -o run -- python3 bench.py --steps 30 --warmup 5 > $O/prof512.log 2>&1 || exit 1
f=$(find $O/prof512 -name "*kernel_stats.csv" | head -1); python3 scripts/kstats.py "$f" > $O/kernels512.txt; cat $O/kernels512.txt
