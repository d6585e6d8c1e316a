# ResNet-50 igemm weight-gradient split heuristic A/B (workgroup target, partial-slab cap)
set -o pipefail
O=gpurun_out/r2x
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_resnet.py > $O/pytest.log 2>&1
rc=$?; tail -1 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
b() { tag=$(echo "$*" | tr ' =' '_-'); timeout -k 10 300 env "$@" python3 bench.py --model resnet50 --steps 15 --warmup 4 > $O/b_$tag.log 2>&1 && echo "$* $(grep '^{' $O/b_$tag.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["median_window_ms_per_step"])')"; }
b DTFE_IG_WTARGET=768 && b DTFE_IG_WPART_MB=32 && b DTFE_IG_WPART_MB=48 && b DTFE_IG_WPART_MB=64 && b DTFE_IG_WPART_MB=24 && \
b DTFE_IG_WTARGET=512 DTFE_IG_WPART_MB=32 && b DTFE_IG_WTARGET=512 DTFE_IG_WPART_MB=48 && b DTFE_IG_WTARGET=640 DTFE_IG_WPART_MB=32 && b DTFE_IG_WPART_MB=32 || exit 1
