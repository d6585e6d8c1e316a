# ResNet-50 B=256 loss sanity (dtfe vs stock torch at the same lr / momentum / step counts)
# and per-layer conv timings.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python3 bench.py --model resnet50 --steps 2 --warmup 0 > gpurun_out/l_dtfe_s2.log 2>&1 &&
timeout -k 10 200 python3 bench.py --model resnet50 --steps 10 --warmup 0 > gpurun_out/l_dtfe_s10.log 2>&1 &&
timeout -k 10 200 python3 bench/stock_torch_resnet.py --arch resnet50 --batch_size 256 --graph --warmup 0 --steps 12 > gpurun_out/l_stock_s12.log 2>&1 &&
timeout -k 10 200 python3 bench/stock_torch_resnet.py --arch resnet50 --batch_size 256 --graph --warmup 0 --steps 60 > gpurun_out/l_stock_s60.log 2>&1 &&
timeout -k 10 300 python3 bench/resnet50_convs.py --batch 256 --reps 10 --no-torch > gpurun_out/r50_convs.log 2>&1
rc=$?
for f in gpurun_out/l_*.log; do echo "$f"; tail -n 1 "$f"; done
cat gpurun_out/r50_convs.log | tail -40
exit $rc
