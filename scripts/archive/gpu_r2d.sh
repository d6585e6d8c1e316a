set -o pipefail
O=gpurun_out/r2d
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gemm_glds_gpu.py tests/test_mnist_cnn_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python3 bench.py --steps 200 --warmup 20 > $O/b_cnn.log 2>&1 && grep '^{' $O/b_cnn.log || exit 1
DTFE_CNN_GLDS=0 timeout -k 10 180 python3 bench.py --steps 200 --warmup 20 > $O/b_cnn_noglds.log 2>&1 && grep '^{' $O/b_cnn_noglds.log | cut -c1-200
DTFE_CNN_BRANCHES=none timeout -k 10 180 python3 bench.py --steps 200 --warmup 20 > $O/b_cnn_nobr.log 2>&1 && grep '^{' $O/b_cnn_nobr.log | cut -c1-200
timeout -k 10 200 python3 bench/cnn_kernels.py --batch_size 1024 --iters 30 > $O/cnn_kernels.txt 2>&1 && cat $O/cnn_kernels.txt
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_cnn -o run -- python3 bench.py --steps 30 --warmup 5 > $O/prof_cnn.log 2>&1
f=$(find $O/prof_cnn -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && python3 scripts/kstats.py "$f" > $O/cnn_kernels_prof.txt && cat $O/cnn_kernels_prof.txt
f=$(find $O/prof_cnn -name "*kernel_trace.csv" | head -1)
[ -n "$f" ] && python3 scripts/timeline.py "$f" conv1c_fwd > $O/cnn_timeline.txt && cat $O/cnn_timeline.txt
timeout -k 10 300 python3 bench/gemm_sweep.py --iters 20 > $O/gemm_sweep.txt 2>&1; cat $O/gemm_sweep.txt
