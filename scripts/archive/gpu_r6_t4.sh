# Round 6: after the BN-fold removal - ResNet tests, the partitioned-ps GPU tests, ResNet-20/50 benches,
# the fp32 CNN kernel table and the reference workloads (LSTM / GAN / autoencoder)
set -o pipefail
O=gpurun_out/${1:-r6t4}
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests/test_resnet.py tests/test_igemm_gpu.py tests/test_igemm_tiles_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu > $O/pytest_resnet.log 2>&1
rc=$?; tail -3 $O/pytest_resnet.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest_resnet.log | head -30; exit $rc; }
timeout -k 10 600 python3 -u -m pytest tests/test_cluster_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "partitioned" > $O/pytest_ps.log 2>&1
rc=$?; tail -3 $O/pytest_ps.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest_ps.log | head -30; }
for m in resnet20 resnet50; do
  timeout -k 10 300 python3 bench.py --model $m --steps 20 --warmup 5 > $O/$m.log 2>&1 || { tail -5 $O/$m.log; exit 1; }
  echo "$m $(grep -o '"value": [0-9.]*' $O/$m.log) $(grep -o '"ms_per_step": [0-9.]*' $O/$m.log)"
done
timeout -k 10 200 python3 bench.py --dtype fp32 --steps 20 --warmup 5 > $O/cnn_fp32.log 2>&1 || { tail -5 $O/cnn_fp32.log; exit 1; }
echo "cnn fp32 $(grep -o '"value": [0-9.]*' $O/cnn_fp32.log) $(grep -o '"ms_per_step": [0-9.]*' $O/cnn_fp32.log)"
timeout -k 10 300 python3 bench/ref_models.py --steps 200 --warmup 20 > $O/ref_models.log 2>&1 || { tail -5 $O/ref_models.log; exit 1; }
cat $O/ref_models.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_fp32 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --dtype fp32 --steps 20 --warmup 5 > $GRAFT_REPO_ROOT/$O/prof_fp32.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$O/prof_fp32.log; exit 1; }
cd $GRAFT_REPO_ROOT
python3 scripts/kstats.py $(ls $O/prof_fp32/*kernel_stats.csv | head -1) > $O/fp32_kstats.txt && cat $O/fp32_kstats.txt
exit $rc
