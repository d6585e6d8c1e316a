# Round 5: weight-gradient pixel target under the grouped (deferred) reduce: DTFE_DIAG iwpx=<mul> / iwpd=<div>
set -o pipefail
O=gpurun_out/r5pxdefer
mkdir -p $O
for rep in 1 2; do
for d in iwpd=1 iwpd=2 iwpd=4; do
  DTFE_DIAG=$d timeout -k 10 200 python3 bench.py --model resnet20 --steps 20 --warmup 5 > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
  echo "$d $(grep -o '"ms_per_step": [0-9.]*' $O/b.log)"
done; done
