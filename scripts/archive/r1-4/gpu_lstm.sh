#!/bin/bash
# LSTM persistent-kernel check + timing on one GPU: tests, split vs single-CU step time, kernel stats.
set -o pipefail
tag=${1:-lstm}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
[ -n "$SKIP_TESTS" ] || timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_models_gpu.py -k lstm > $out/pytest.txt 2>&1 || { tail -40 $out/pytest.txt; exit 1; }
tail -3 $out/pytest.txt
DTFE_LSTM_SPLIT=0 timeout -k 10 120 python -u bench/ref_models.py --models lstm --steps 300 --warmup 30 > $out/ref_split0.txt 2>&1 && cat $out/ref_split0.txt | tail -2 &&
DTFE_LSTM_SPLIT=1 timeout -k 10 120 python -u bench/ref_models.py --models lstm --steps 300 --warmup 30 > $out/ref_split1.txt 2>&1 && cat $out/ref_split1.txt | tail -2 &&
DTFE_LSTM_SPLIT=0 timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof0 -o run -- python3 bench/ref_models.py --models lstm --steps 100 --warmup 10 > $out/prof0.log 2>&1 &&
f=$(find $out/prof0 -name "*kernel_stats.csv" | head -1) && python3 scripts/kstats.py "$f" > $out/kernels0.txt && cat $out/kernels0.txt &&
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- python3 bench/ref_models.py --models lstm --steps 100 --warmup 10 > $out/prof.log 2>&1 &&
f=$(find $out/prof -name "*kernel_stats.csv" | head -1) && python3 scripts/kstats.py "$f" > $out/kernels.txt && cat $out/kernels.txt
