# Head weight gradient as the grouped fc-backward launch's first piece (4-column body, 84 VGPRs)
# vs its own launch before the group: tests (group bitwise vs separate launches; CNN numerics with
# the piece in the group) + step A/B + timeline.
set -o pipefail
O=gpurun_out/r3ze
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gemm_glds_gpu.py -x -q -m gpu -k "group" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_g.log 2>&1
rc=$?; tail -1 $O/pytest_g.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest_g.log | head -20; exit $rc; }
DTFE_CNN_HEAD_IN_GROUP=1 timeout -k 10 300 python3 -u -m pytest tests/test_mnist_cnn_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_c.log 2>&1
rc=$?; tail -1 $O/pytest_c.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest_c.log | head -20; exit $rc; }
for r in 1 2 3; do
  for v in 0 1; do
    DTFE_CNN_HEAD_IN_GROUP=$v timeout -k 10 120 python3 bench.py > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
    echo "head_in_group=$v $(grep -o '"ms_per_step": [0-9.]*' $O/b.log)"
  done
done
export DTFE_CNN_HEAD_IN_GROUP=1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 30 --warmup 5 > $O/prof.log 2>&1 || exit 1
f=$(find $O/prof -name "*kernel_trace.csv" | head -1)
[ -n "$f" ] && python3 scripts/timeline.py "$f" conv1c_fwd > $O/timeline.txt && cat $O/timeline.txt
exit 0
