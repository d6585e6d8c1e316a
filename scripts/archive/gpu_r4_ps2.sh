# Round-4: fused ps replies + fence-free hand-offs: cluster/ps GPU tests, 1+1 bench, merged timeline
set -o pipefail
O=gpurun_out/r4ps2
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_cluster_gpu.py > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -30; exit $rc; }
for i in 1 2; do
  timeout -k 10 240 python3 bench.py --mode ps --gpus 1 --steps 200 --warmup 20 > $O/ps11_$i.log 2>&1 || { tail -5 $O/ps11_$i.log; exit 1; }
  grep '^{' $O/ps11_$i.log | cut -c1-220
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
DTFE_PROFILE_EXIT=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_ps -o run_%pid% -- python3 bench.py --mode ps --gpus 1 --steps 40 --warmup 10 > $O/prof_ps.log 2>&1 || { tail -5 $O/prof_ps.log; exit 1; }
python3 scripts/ps_timeline.py $O/prof_ps > $O/ps_timeline.txt 2>&1; tail -30 $O/ps_timeline.txt
