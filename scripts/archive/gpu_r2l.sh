# tall-K LSTM kernel gradient + optimizer chunk A/B (one GPU)
set -o pipefail
O=gpurun_out/r2l
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_models_gpu.py tests/test_kernels_gpu.py -k "lstm or tallk or optim or apply" > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -20; exit $rc; }
timeout -k 10 120 python3 bench/lstm_wgrad_sweep.py > $O/lstm_wgrad.txt 2>&1; cat $O/lstm_wgrad.txt
timeout -k 10 200 python3 bench/ref_models.py --steps 300 --warmup 30 > $O/ref_models.txt 2>&1 && grep '^{' $O/ref_models.txt || exit 1
b() { tag=$(echo "$*" | tr ' =' '_-'); timeout -k 10 180 env "$@" python3 bench.py --steps 300 --warmup 30 > $O/b_$tag.log 2>&1 && echo "$* $(grep '^{' $O/b_$tag.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["median_window_ms_per_step"])')"; }
b DTFE_OPT_CHUNK=8192 && b DTFE_OPT_CHUNK=4096 && b DTFE_OPT_CHUNK=2048 && b DTFE_OPT_CHUNK=16384 || exit 1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_lstm -o run -- python3 bench/ref_models.py --models lstm --steps 100 --warmup 10 > $O/prof_lstm.log 2>&1 || exit 1
f=$(find $O/prof_lstm -name "*kernel_trace.csv" | head -1); python3 scripts/trace_summary.py "$f" seq_stage > $O/lstm_trace.txt 2>&1; cat $O/lstm_trace.txt
