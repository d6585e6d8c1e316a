# ResNet-50: forward/dgrad split-K workgroup target A/B (with the tuned weight-gradient splits), + R20 / CNN check
set -o pipefail
O=gpurun_out/r2y
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_resnet.py tests/test_imgconv.py tests/test_norm_gpu.py > $O/pytest.log 2>&1
rc=$?; tail -1 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head; exit $rc; }
b() { tag=$(echo "$*" | tr ' =' '_-'); timeout -k 10 300 env "$@" python3 bench.py --model resnet50 --steps 15 --warmup 4 > $O/b_$tag.log 2>&1 && echo "$* $(grep '^{' $O/b_$tag.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["median_window_ms_per_step"])')"; }
b DTFE_IG_TBLOCKS=240 && b DTFE_IG_TBLOCKS=480 && b DTFE_IG_TBLOCKS=720 && b DTFE_IG_TBLOCKS=1024 && b DTFE_IG_TBLOCKS=160 && b DTFE_IG_TBLOCKS=240 || exit 1
timeout -k 10 240 python3 bench.py --model resnet20 --steps 100 --warmup 10 > $O/b_r20.log 2>&1 && grep '^{' $O/b_r20.log | cut -c1-200
