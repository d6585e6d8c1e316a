# CNN backward schedule variants + LSTM kernel-gradient GEMM sweep (one GPU)
set -o pipefail
O=gpurun_out/r2i
mkdir -p $O
b() { tag=$(echo "$*" | tr ' =' '_-'); timeout -k 10 180 env "$@" python3 bench.py --steps 300 --warmup 30 > $O/b_$tag.log 2>&1 && echo "$* $(grep '^{' $O/b_$tag.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["median_window_ms_per_step"])')"; }
timeout -k 10 120 python3 bench/lstm_wgrad_sweep.py > $O/lstm_wgrad.txt 2>&1; cat $O/lstm_wgrad.txt
b DTFE_X=base && b DTFE_CNN_HEAD_WHERE=last && b DTFE_CNN_HEAD_WHERE=c2 && b DTFE_CNN_EARLY_JOIN=1 && \
b DTFE_CNN_HEAD_WHERE=c2 DTFE_CNN_EARLY_JOIN=1 && b DTFE_CNN_HEAD_WHERE=last DTFE_CNN_EARLY_JOIN=1 && b DTFE_X=base2 || exit 1
