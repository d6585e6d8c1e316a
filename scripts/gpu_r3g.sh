# MNIST CNN conv2 kernels: phase ablation (DTFE_IC_DIAG) of the current fwd / dgrad kernels, per-op table,
# PMC counter passes over the per-op bench
set -o pipefail
O=gpurun_out/r3g
mkdir -p $O
for d in 0 1 2 4 5 7; do
  echo "DIAG=$d"
  DTFE_IC_DIAG=$d timeout -k 10 120 python3 bench/conv2_scale.py > $O/diag_$d.txt 2>&1 || { tail -3 $O/diag_$d.txt; exit 1; }
  grep "B=" $O/diag_$d.txt
done
timeout -k 10 200 python3 bench/cnn_kernels.py --batch_size 1024 --iters 50 > $O/ops.txt 2>&1 || { tail -3 $O/ops.txt; exit 1; }
grep -v amdgpu.ids $O/ops.txt
bash scripts/pmc.sh r3g_cnn -- python3 bench/cnn_kernels.py --batch_size 1024 --iters 5 > $O/pmc.txt 2>&1 || { tail -5 $O/pmc.txt; exit 1; }
grep -E "^kernel|imgconv|imgwgrad|conv1c|gemm_glds|head_|apply_grad" $O/pmc.txt | cut -c1-400
