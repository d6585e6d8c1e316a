# usage: bash scripts/profile.sh <tag> [bench args...]
set -o pipefail
tag=$1; shift
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/prof_$tag
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -o run -- python3 bench.py "$@" > gpurun_out/prof_$tag/stdout.log 2>&1
rc=$?
echo "rocprof exit $rc"
find gpurun_out/prof_$tag -name "*kernel_stats.csv" | head -3
f=$(find gpurun_out/prof_$tag -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && head -25 "$f"
exit $rc
