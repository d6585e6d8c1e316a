# ResNet-20: workgroups of the persistent weight-gradient kernel (images per workgroup) A/B
set -o pipefail
O=gpurun_out/r2t
mkdir -p $O
b() { tag=$(echo "$*" | tr ' =' '_-'); timeout -k 10 180 env "$@" python3 bench.py --model resnet20 --steps 100 --warmup 10 > $O/b_$tag.log 2>&1 && echo "$* $(grep '^{' $O/b_$tag.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["median_window_ms_per_step"])')"; }
for rep in 1 2; do b DTFE_IMGW_BLOCKS=0 && b DTFE_IMGW_BLOCKS=128 && b DTFE_IMGW_BLOCKS=64 && b DTFE_IMGW_BLOCKS=32 || exit 1; done
