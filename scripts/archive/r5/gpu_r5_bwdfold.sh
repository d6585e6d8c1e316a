# Round 5: ResNet-20 bn1 backward formed on conv1's gradient loads + 4x2 waves for <= 8x8 maps:
# numerics, then same-box step A/B (HEAD library; DTFE_DIAG icr=128 = old small-map config;
# DTFE_R20_BWD_FOLD=0 = materialised bn1 backward apply)
set -o pipefail
O=gpurun_out/r5bwdfold
mkdir -p $O
AB=distributed-tensorflow-examples_amd/_C/ab/libdtfe_kernels.so
timeout -k 10 120 python3 bench/resnet20_kernels.py --only "s3 conv" > $O/k_new.txt 2>&1 || { tail -5 $O/k_new.txt; exit 1; }
DTFE_DIAG=icr=128 timeout -k 10 120 python3 bench/resnet20_kernels.py --only "s3 conv" > $O/k_cfg.txt 2>&1 || { tail -5 $O/k_cfg.txt; exit 1; }
echo "== new"; grep -v amdgpu.ids $O/k_new.txt; echo "== icr=128"; grep -v amdgpu.ids $O/k_cfg.txt
for rep in 1 2 3; do
  unset DTFE_KERNEL_LIB DTFE_DIAG DTFE_R20_BWD_FOLD
  timeout -k 10 200 python3 bench.py --model resnet20 --steps 20 --warmup 5 > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
  echo "all-new $(grep -o '"ms_per_step": [0-9.]*' $O/b.log)"
  DTFE_DIAG=icr=128 timeout -k 10 200 python3 bench.py --model resnet20 --steps 20 --warmup 5 > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
  echo "old-s3cfg $(grep -o '"ms_per_step": [0-9.]*' $O/b.log)"
  DTFE_R20_BWD_FOLD=0 timeout -k 10 200 python3 bench.py --model resnet20 --steps 20 --warmup 5 > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
  echo "no-bwdfold $(grep -o '"ms_per_step": [0-9.]*' $O/b.log)"
  DTFE_DIAG=icr=128 DTFE_R20_BWD_FOLD=0 timeout -k 10 200 python3 bench.py --model resnet20 --steps 20 --warmup 5 > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
  echo "both-off $(grep -o '"ms_per_step": [0-9.]*' $O/b.log)"
done
