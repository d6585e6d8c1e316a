# shortcut gradient folded into the whole-image data-gradient epilogue: conv / ResNet tests, ResNet-20 A/B
set -o pipefail
O=gpurun_out/r3a
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_imgconv.py tests/test_resnet.py tests/test_norm_gpu.py > $O/pytest.log 2>&1
rc=$?; tail -1 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -20; exit $rc; }
b() { tag=$(echo "$*" | tr ' =' '_-'); timeout -k 10 240 env "$@" python3 bench.py --model resnet20 --steps 100 --warmup 10 > $O/b_$tag.log 2>&1 && echo "$* $(grep '^{' $O/b_$tag.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["median_window_ms_per_step"])')"; }
for rep in 1 2; do b DTFE_R50_SHORTCUT_FUSE=1 && b DTFE_R50_SHORTCUT_FUSE=0 || exit 1; done
