# Re-tune the two concurrent weight-gradient grids under the final schedule (head in the group):
# conv2 wgrad workgroups (DTFE_CNN_C2_BLOCKS) and conv1 wgrad workgroups (DTFE_C1W_GRID).
set -o pipefail
O=gpurun_out/r3zg2
mkdir -p $O
for r in 1 2 3; do
  for v in d w320 w384 w448 w512; do
    unset DTFE_CNN_C2_BLOCKS DTFE_C1W_GRID
    case $v in w384) export DTFE_C1W_GRID=384;; w448) export DTFE_C1W_GRID=448;; w512) export DTFE_C1W_GRID=512;;
               w320) export DTFE_C1W_GRID=320;; esac
    timeout -k 10 120 python3 bench.py > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
    echo "$v $(grep -o '"ms_per_step": [0-9.]*' $O/b.log)"
  done
done
exit 0
