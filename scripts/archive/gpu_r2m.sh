# Round-2 BASELINE refresh on one GPU: ResNet-20 / ResNet-50 / CNN benches, PS 1+2 and a 1 ps + 8 worker
# rehearsal (all ranks sharing the one GPU), then the 2-rank all-reduce rehearsal (gloo + IPC).
set -o pipefail
O=gpurun_out/r2m
mkdir -p $O
timeout -k 10 180 python3 bench.py --steps 300 --warmup 30 > $O/b_cnn.log 2>&1 && grep '^{' $O/b_cnn.log | cut -c1-300 &&
timeout -k 10 240 python3 bench.py --model resnet20 --steps 50 --warmup 10 > $O/b_r20.log 2>&1 && grep '^{' $O/b_r20.log | cut -c1-300 &&
timeout -k 10 300 python3 bench.py --model resnet50 --steps 20 --warmup 5 > $O/b_r50.log 2>&1 && grep '^{' $O/b_r50.log | cut -c1-300 &&
timeout -k 10 240 python3 bench.py --mode ps --gpus 2 --steps 50 --warmup 5 > $O/b_ps2.log 2>&1 && grep '^{' $O/b_ps2.log | cut -c1-300 &&
timeout -k 10 300 python3 bench.py --gpus 2 --backend gloo --comm ipc --steps 50 --warmup 5 > $O/b_ar2.log 2>&1 && grep '^{' $O/b_ar2.log | cut -c1-600 &&
timeout -k 10 400 python3 bench.py --mode ps --gpus 8 --steps 30 --warmup 5 > $O/b_ps8.log 2>&1 && grep '^{' $O/b_ps8.log | cut -c1-600
