# Round-5 baseline on the round-4 tree: CNN driver shape with / without the pre-warm, ResNet-50 and
# ResNet-20 benches, the ResNet-50 BatchNorm roofline, ResNet-20 and ResNet-50 kernel tables.
set -o pipefail
O=gpurun_out/${1:-r5base}
mkdir -p $O
for pw in 150 0; do
  timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --prewarm_ms $pw > $O/cnn_pw$pw.log 2>&1 || { tail -5 $O/cnn_pw$pw.log; exit 1; }
  echo "cnn prewarm=$pw $(grep -o '"value": [0-9.]*' $O/cnn_pw$pw.log) $(grep -o '"ms_per_step": [0-9.]*' $O/cnn_pw$pw.log)"
done
timeout -k 10 300 python3 bench.py --model resnet50 --steps 20 --warmup 5 > $O/r50.log 2>&1 || { tail -5 $O/r50.log; exit 1; }
echo "r50 $(grep -o '"value": [0-9.]*' $O/r50.log) $(grep -o '"ms_per_step": [0-9.]*' $O/r50.log)"
timeout -k 10 200 python3 bench.py --model resnet20 --steps 50 --warmup 10 > $O/r20.log 2>&1 || { tail -5 $O/r20.log; exit 1; }
echo "r20 $(grep -o '"value": [0-9.]*' $O/r20.log) $(grep -o '"ms_per_step": [0-9.]*' $O/r20.log)"
timeout -k 10 300 python3 bench/bn_roofline.py > $O/bn_roofline.txt 2>&1 || { tail -5 $O/bn_roofline.txt; exit 1; }
tail -3 $O/bn_roofline.txt
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_r20 -o run -- python3 bench.py --model resnet20 --steps 20 --warmup 5 --prewarm_ms 0 > $O/prof_r20.log 2>&1 || { tail -5 $O/prof_r20.log; exit 1; }
f=$(find $O/prof_r20 -name "*kernel_stats.csv" | head -1); python3 scripts/kstats.py "$f" > $O/r20_kernels.txt; tail -1 $O/r20_kernels.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_r50 -o run -- python3 bench.py --model resnet50 --steps 8 --warmup 5 --prewarm_ms 0 > $O/prof_r50.log 2>&1 || { tail -5 $O/prof_r50.log; exit 1; }
f=$(find $O/prof_r50 -name "*kernel_stats.csv" | head -1); python3 scripts/kstats.py "$f" > $O/r50_kernels.txt; tail -1 $O/r50_kernels.txt
