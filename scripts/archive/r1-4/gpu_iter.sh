# One iteration on one GPU: kernel/model tests, headline bench, reference workloads, and
# rocprofv3 kernel stats + step timelines (CNN, GAN).  Usage: bash scripts/gpu_iter.sh <tag>
set -o pipefail
tag=${1:-iter}
O=gpurun_out/$tag
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest tests/test_kernels_gpu.py tests/test_mnist_cnn_gpu.py tests/test_imgconv.py tests/test_models_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -30; exit $rc; }
timeout -k 10 180 python3 bench.py --steps 300 --warmup 30 > $O/b_cnn.log 2>&1 && grep '^{' $O/b_cnn.log | cut -c1-200 || exit 1
DTFE_CNN_HEAD_GEMM=1 timeout -k 10 180 python3 bench.py --steps 300 --warmup 30 > $O/b_cnn_headgemm.log 2>&1 && grep '^{' $O/b_cnn_headgemm.log | cut -c1-200 || exit 1
timeout -k 10 200 python3 bench/ref_models.py --steps 300 --warmup 30 > $O/ref_models.txt 2>&1 && grep '^{' $O/ref_models.txt || exit 1
DTFE_GEMM_SMALL=0 timeout -k 10 200 python3 bench/ref_models.py --models gan,encoder --steps 300 --warmup 30 > $O/ref_models_nosmall.txt 2>&1 && grep '^{' $O/ref_models_nosmall.txt || exit 1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 30 --warmup 5 > $O/prof.log 2>&1 || exit 1
f=$(find $O/prof -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && python3 scripts/kstats.py "$f" > $O/kernels.txt && cat $O/kernels.txt
f=$(find $O/prof -name "*kernel_trace.csv" | head -1)
[ -n "$f" ] && python3 scripts/timeline.py "$f" conv1c_fwd > $O/timeline.txt && cat $O/timeline.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_gan -o run -- python3 bench/ref_models.py --models gan --steps 50 --warmup 5 > $O/prof_gan.log 2>&1 || exit 1
f=$(find $O/prof_gan -name "*kernel_trace.csv" | head -1)
[ -n "$f" ] && python3 scripts/trace_summary.py "$f" uniform_fill > $O/gan_trace.txt 2>&1; cat $O/gan_trace.txt
exit 0
