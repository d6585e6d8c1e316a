# Round 5: ResNet-20 stem - weight gradient images-per-workgroup sweep (DTFE_DIAG iw1=<n>) and the
# forward's LDS-staged epilogue (DTFE_DIAG ic1=1: the old scattered stores)
set -o pipefail
O=gpurun_out/r5stemwg
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_imgconv.py tests/test_resnet.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -30; exit $rc; }
for n in 0 1 4 8; do
  DTFE_DIAG=iw1=$n timeout -k 10 120 python3 bench/resnet20_kernels.py --only "stem" > $O/k$n.txt 2>&1 || { tail -5 $O/k$n.txt; exit 1; }
  echo "== ipb=$n"; grep -v amdgpu.ids $O/k$n.txt
done
DTFE_DIAG=ic1=1 timeout -k 10 120 python3 bench/resnet20_kernels.py --only "stem" > $O/kold.txt 2>&1 || { tail -5 $O/kold.txt; exit 1; }
echo "== ic1=1"; grep -v amdgpu.ids $O/kold.txt
