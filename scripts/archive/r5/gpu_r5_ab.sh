# Round 5 same-box A/B: the kernel library at HEAD vs an --ab build (csrc/build.py --ab REV FILE...),
# alternating: write roofline, ResNet-50 conv table, ResNet-50 bench
set -o pipefail
O=gpurun_out/${1:-r5ab}
mkdir -p $O
AB=distributed-tensorflow-examples_amd/_C/ab/libdtfe_kernels.so
for r in 1 2; do
  for v in new old; do
    if [ $v = old ]; then export DTFE_KERNEL_LIB=$AB; else unset DTFE_KERNEL_LIB; fi
    timeout -k 10 200 python3 bench/write_roofline.py > $O/wr_${v}_$r.txt 2>&1 || { tail -5 $O/wr_${v}_$r.txt; exit 1; }
    echo "== $v $r"; grep conv $O/wr_${v}_$r.txt
    timeout -k 10 300 python3 bench.py --model resnet50 --steps 20 --warmup 5 > $O/r50_${v}_$r.log 2>&1 || { tail -5 $O/r50_${v}_$r.log; exit 1; }
    echo "r50 $v $r $(grep -o '"value": [0-9.]*' $O/r50_${v}_$r.log) $(grep -o '"ms_per_step": [0-9.]*' $O/r50_${v}_$r.log)"
  done
done
for v in new old; do
  if [ $v = old ]; then export DTFE_KERNEL_LIB=$AB; else unset DTFE_KERNEL_LIB; fi
  timeout -k 10 300 python3 bench/resnet50_convs.py --batch 256 --reps 10 --no-torch > $O/convs_$v.txt 2>&1 || { tail -5 $O/convs_$v.txt; exit 1; }
  echo "== convs $v"; tail -1 $O/convs_$v.txt
done
unset DTFE_KERNEL_LIB
timeout -k 10 200 python3 bench.py --dtype fp32 --steps 50 --warmup 5 > $O/cnn_fp32.log 2>&1 || { tail -5 $O/cnn_fp32.log; exit 1; }
echo "cnn fp32 $(grep -o '"value": [0-9.]*' $O/cnn_fp32.log) $(grep -o '"ms_per_step": [0-9.]*' $O/cnn_fp32.log)"
timeout -k 10 200 python3 bench/stock_torch_cnn.py --dtype fp32 --fused --steps 50 > $O/stock_fp32.log 2>&1 || { tail -5 $O/stock_fp32.log; exit 1; }
timeout -k 10 200 python3 bench/stock_torch_cnn.py --dtype fp32 --graph --steps 50 > $O/stock_fp32_graph.log 2>&1 || { tail -5 $O/stock_fp32_graph.log; exit 1; }
grep -h '^{' $O/stock_fp32.log $O/stock_fp32_graph.log
timeout -k 10 300 python3 bench/ref_models.py > $O/ref_models.log 2>&1 || { tail -5 $O/ref_models.log; exit 1; }
grep -v amdgpu $O/ref_models.log | tail -6
