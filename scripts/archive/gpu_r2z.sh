# ResNet-20: persistent conv wave grid A/B (DTFE_IC_WAVES: 16 = 8x2 waves (default), 8 = 4x2, 4 = 4x1)
set -o pipefail
O=gpurun_out/r2z
mkdir -p $O
b() { tag=$(echo "$*" | tr ' =' '_-'); timeout -k 10 240 env "$@" python3 bench.py --model resnet20 --steps 100 --warmup 10 > $O/b_$tag.log 2>&1 && echo "$* $(grep '^{' $O/b_$tag.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["median_window_ms_per_step"])')"; }
for rep in 1 2; do b DTFE_IC_WAVES=16 && b DTFE_IC_WAVES=8 && b DTFE_IC_WAVES=4 || exit 1; done
