# Round 5: ResNet-50 kernel tables with the bn1 / bn2 applies folded (DTFE_R5_FOLD=1) and materialised (0)
set -o pipefail
O=gpurun_out/${1:-r5foldprof}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for f in 1 0; do
  DTFE_R5_FOLD=$f timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_f$f -o run -- python3 bench.py --model resnet50 --steps 8 --warmup 5 --prewarm_ms 0 > $O/prof_f$f.log 2>&1 || { tail -5 $O/prof_f$f.log; exit 1; }
  f2=$(find $O/prof_f$f -name "*kernel_stats.csv" | head -1); python3 scripts/kstats.py "$f2" > $O/r50_kernels_f$f.txt; tail -1 $O/r50_kernels_f$f.txt
done
