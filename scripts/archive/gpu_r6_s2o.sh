# Round 6 (session 2): conv1 forward grid (images per workgroup: 1 / 2 / 4, next image's gather prefetched)
set -o pipefail
O=gpurun_out/${1:-r6s2o}
mkdir -p $O
for r in 1 2; do
for g in 1024 512 256; do
  DTFE_DIAG=c1g=$g timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 > $O/c1g_${g}_$r.log 2>&1 || { tail -5 $O/c1g_${g}_$r.log; exit 1; }
  echo "c1g=$g $(grep -o '"ms_per_step": [0-9.]*' $O/c1g_${g}_$r.log)"
done
done
for g in 1024 512 256; do
  DTFE_DIAG=c1g=$g timeout -k 10 120 python3 bench/cnn_kernels.py --only conv1_fwd --iters 50 > $O/k_$g.log 2>&1 || { tail -5 $O/k_$g.log; exit 1; }
  echo "c1g=$g $(grep conv1_fwd $O/k_$g.log)"
done
