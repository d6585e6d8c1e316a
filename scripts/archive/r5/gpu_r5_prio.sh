# Round 5: MNIST CNN conv2-wgrad branch stream priority A/B (0 = default, -1 = high)
set -o pipefail
O=gpurun_out/r5prio
mkdir -p $O
for rep in 1 2; do
for pr in 0 -1; do
for pw in 150 0; do
  DTFE_CNN_C2_PRIO=$pr timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --prewarm_ms $pw > $O/c.log 2>&1 || { tail -5 $O/c.log; exit 1; }
  echo "prio=$pr pw=$pw $(grep -o '"ms_per_step": [0-9.]*' $O/c.log)"
done; done; done
