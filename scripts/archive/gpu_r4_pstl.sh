# Round-4: 1 ps + 1 worker kernel timeline (both processes on one GPU)
set -o pipefail
O=gpurun_out/${1:-r4pstl}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
DTFE_PROFILE_EXIT=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_ps -o run_%pid% -- python3 bench.py --mode ps --gpus 1 --steps 40 --warmup 10 > $O/prof_ps.log 2>&1 || { tail -5 $O/prof_ps.log; exit 1; }
python3 scripts/ps_timeline.py $O/prof_ps > $O/ps_timeline.txt 2>&1; cat $O/ps_timeline.txt
