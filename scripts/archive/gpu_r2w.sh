# multi-rank rehearsals on ONE GPU (ranks share the card; gloo control plane + IPC all-reduce):
# CNN at 4 ranks, ResNet-20 at 2 ranks - W=4 kernel instantiation, bucket routing, replica agreement
set -o pipefail
O=gpurun_out/r2w
mkdir -p $O
timeout -k 10 400 python3 bench.py --gpus 4 --backend gloo --comm ipc --steps 30 --warmup 5 > $O/b_cnn4.log 2>&1 && grep '^{' $O/b_cnn4.log | cut -c1-900 &&
timeout -k 10 400 python3 bench.py --model resnet20 --gpus 2 --backend gloo --comm ipc --steps 20 --warmup 5 > $O/b_r20x2.log 2>&1 && grep '^{' $O/b_r20x2.log | cut -c1-900 || exit 1
b() { tag=$(echo "$*" | tr ' =' '_-'); timeout -k 10 180 env "$@" python3 bench.py --steps 300 --warmup 30 > $O/b_$tag.log 2>&1 && echo "$* $(grep '^{' $O/b_$tag.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["median_window_ms_per_step"])')"; }
for rep in 1 2; do b DTFE_CNN_C2_BLOCKS=128 && b DTFE_CNN_C2_BLOCKS=64 && b DTFE_CNN_C2_BLOCKS=96 && b DTFE_CNN_C2_BLOCKS=192 && b DTFE_CNN_C2_BLOCKS=256 || exit 1; done
