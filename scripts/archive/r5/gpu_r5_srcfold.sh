# Round 5: ResNet-20 bn1 apply formed by conv2's whole-image kernels (BN.src_fold): numerics + A/B
set -o pipefail
O=gpurun_out/r5srcfold
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_imgconv.py tests/test_resnet.py tests/test_norm_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -30; exit $rc; }
timeout -k 10 120 python3 bench/resnet20_kernels.py --only "conv2 fwd,conv2 wgrad,bn1 apply" > $O/k.txt 2>&1 || { tail -5 $O/k.txt; exit 1; }
grep -v amdgpu.ids $O/k.txt
for rep in 1 2; do
for f in 1 0; do
  DTFE_R20_SRC_FOLD=$f timeout -k 10 200 python3 bench.py --model resnet20 --steps 20 --warmup 5 > $O/bench$f.log 2>&1 || { tail -5 $O/bench$f.log; exit 1; }
  echo "fold=$f $(grep -o '"ms_per_step": [0-9.]*' $O/bench$f.log)"
done; done
