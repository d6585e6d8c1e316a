# per-bucket reply snapshots on the ps: PS tests, PS bench, per-process PS kernel traces; ResNet-50 step kernel table
set -o pipefail
O=gpurun_out/r3f
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_cluster_gpu.py > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -20; exit $rc; }
for i in 1 2; do
  timeout -k 10 200 python3 bench.py --mode ps --gpus 1 --steps 200 --warmup 20 > $O/ps_$i.log 2>&1 || exit 1
  echo "ps $(grep '^{' $O/ps_$i.log | cut -c1-250)"
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
DTFE_PROFILE_EXIT=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_ps -o run_%pid% -- python3 bench.py --mode ps --gpus 1 --steps 40 --warmup 10 > $O/prof_ps.log 2>&1 || exit 1
find $O/prof_ps -name "*kernel_trace.csv"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_r50 -o run -- python3 bench.py --model resnet50 --steps 8 --warmup 5 > $O/prof_r50.log 2>&1 || exit 1
find $O/prof_r50 -name "*kernel_stats.csv"
