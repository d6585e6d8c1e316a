# igemm 8-wave pipelined tiles: tile-equivalence tests, per-layer ResNet-50 conv table (B=256) with the
# 8-wave kernel on and off, and the ResNet-50 B=256 step both ways.
set -o pipefail
O=gpurun_out/r3igemm
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_igemm_tiles_gpu.py tests/test_resnet.py > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -20; exit $rc; }
timeout -k 10 400 python3 bench/resnet50_convs.py --batch 256 --reps 10 > $O/convs_8w.txt 2>&1 || exit 1
DTFE_IG_8W=0 timeout -k 10 400 python3 bench/resnet50_convs.py --batch 256 --reps 10 --no-torch > $O/convs_4w.txt 2>&1 || exit 1
cat $O/convs_8w.txt; tail -2 $O/convs_4w.txt
for v in 1 0 1 0; do
  DTFE_IG_8W=$v timeout -k 10 300 python3 bench.py --model resnet50 --steps 20 --warmup 5 > $O/r50_$v.log 2>&1 || exit 1
  echo "8w=$v $(grep '^{' $O/r50_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["last_loss"])')"
done
