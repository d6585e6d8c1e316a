# Round-4: ResNet-50 step timeline (the tail: which stream finishes last)
set -o pipefail
O=gpurun_out/r4r50tl
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 bench.py --model resnet50 --steps 6 --warmup 4 > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
f=$(find $O/prof -name "*kernel_trace.csv" | head -1); python3 scripts/timeline.py "$f" stem_fwd > $O/timeline.txt; tail -45 $O/timeline.txt
