# Round 2, first GPU pass: the GPU suite (incl. the bench self-launcher test), the headline
# bench, ResNet-50 at B=256 and B=64, ResNet-20, and a kernel profile of ResNet-50 B=256.
set -o pipefail
O=gpurun_out/r2a
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python3 bench.py --steps 200 --warmup 20 > $O/b_cnn.log 2>&1 && grep '^{' $O/b_cnn.log &&
timeout -k 10 300 python3 bench.py --model resnet50 --steps 20 --warmup 5 > $O/b_r50_256.log 2>&1 && grep '^{' $O/b_r50_256.log &&
timeout -k 10 300 python3 bench.py --model resnet50 --batch_size 64 --steps 20 --warmup 5 > $O/b_r50_64.log 2>&1 && grep '^{' $O/b_r50_64.log &&
timeout -k 10 200 python3 bench.py --model resnet20 --steps 50 --warmup 10 > $O/b_r20.log 2>&1 && grep '^{' $O/b_r20.log || exit $?
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_r50 -o run -- python3 bench.py --model resnet50 --steps 10 --warmup 3 > $O/prof_r50.log 2>&1
rc=$?
f=$(find $O/prof_r50 -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && python3 scripts/kstats.py "$f" > $O/r50_b256_kernels.txt && head -40 $O/r50_b256_kernels.txt
exit $rc
