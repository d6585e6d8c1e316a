# fused Adam apply: work-item size and load depth A/B on the CNN step (one GPU)
set -o pipefail
O=gpurun_out/r2r
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "optim or apply" > $O/pytest.log 2>&1
rc=$?; tail -1 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
b() { tag=$(echo "$*" | tr ' =' '_-'); timeout -k 10 180 env "$@" python3 bench.py --steps 300 --warmup 30 > $O/b_$tag.log 2>&1 && echo "$* $(grep '^{' $O/b_$tag.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["median_window_ms_per_step"])')"; }
for rep in 1 2; do
b DTFE_OPT_CHUNK=8192 && b DTFE_OPT_CHUNK=16384 && b DTFE_OPT_CHUNK=32768 && b DTFE_OPT_DEEP=1 DTFE_OPT_CHUNK=16384 && b DTFE_OPT_DEEP=1 DTFE_OPT_CHUNK=32768 || exit 1
done
