# eager multi-stream launches vs hipGraph replay for the CNN step (host launch overhead vs graph queue edges)
set -o pipefail
O=gpurun_out/r2v
mkdir -p $O
b() { tag=$(echo "$*" | tr ' =' '_-'); timeout -k 10 180 env "$@" python3 bench.py --steps 300 --warmup 30 > $O/b_$tag.log 2>&1 && echo "$* $(grep '^{' $O/b_$tag.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["median_window_ms_per_step"])')"; }
for rep in 1 2; do b DTFE_GRAPHS=1 && b DTFE_GRAPHS=0 || exit 1; done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
DTFE_GRAPHS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_cnn -o run -- python3 bench.py --steps 30 --warmup 5 > $O/prof_cnn.log 2>&1 || exit 1
f=$(find $O/prof_cnn -name "*kernel_trace.csv" | head -1); python3 scripts/timeline.py "$f" conv1c_fwd > $O/cnn_timeline.txt; cat $O/cnn_timeline.txt
