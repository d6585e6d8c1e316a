# Round 5: LDS-staged conv epilogue + one-column wave grid for N=16 (ResNet-20): numerics, kernels, step
set -o pipefail
O=gpurun_out/r5stage
mkdir -p $O
timeout -k 10 120 /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 bench/atomic_contention.hip -o $O/atomic_contention && timeout -k 10 60 $O/atomic_contention > $O/atomic.txt 2>&1 || { tail -5 $O/atomic.txt; exit 1; }
cat $O/atomic.txt; rm -f $O/atomic_contention
timeout -k 10 300 python3 -u -m pytest tests/test_imgconv.py tests/test_resnet.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -30; exit $rc; }
for d in 0 16 32 48; do
  echo "== icr=$d"
  DTFE_DIAG=icr=$d timeout -k 10 120 python3 bench/resnet20_kernels.py --only "conv1 fwd,conv2 dgrad,conv1 dgrad" > $O/k$d.txt 2>&1 || { tail -5 $O/k$d.txt; exit 1; }
  grep -v amdgpu.ids $O/k$d.txt
done
timeout -k 10 200 python3 bench.py --model resnet20 --steps 20 --warmup 5 > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*' $O/bench.log
DTFE_DIAG=icr=48 timeout -k 10 200 python3 bench.py --model resnet20 --steps 20 --warmup 5 > $O/bench_old.log 2>&1 || { tail -5 $O/bench_old.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*' $O/bench_old.log
