# Warm-up ramp of a fresh bench process: per-kernel durations over the first vs the last steps.
set -o pipefail
O=gpurun_out/r3zd
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 bench.py --steps 200 --warmup 5 > $O/prof.log 2>&1 || exit 1
f=$(find $O/prof -name "*kernel_trace.csv" | head -1)
python3 scripts/ramp_kernels.py "$f" > $O/ramp.txt && cat $O/ramp.txt
grep -o '"window_ms_per_step": \[[^]]*\]' $O/prof.log
exit 0
