# Round 6: async-PS rows (ranks time-sharing one GPU): 1+1, 1+2, 1+8, 2+8 partitioned (fc1 split over both ps)
set -o pipefail
O=gpurun_out/${1:-r6ps}
mkdir -p $O
row() {
  local tag=$1; shift
  timeout -k 10 300 python3 bench.py "$@" > $O/$tag.log 2>&1 || { tail -5 $O/$tag.log; exit 1; }
  echo "$tag $(tail -1 $O/$tag.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d["median_window_ms_per_step"], d["window_ms_per_step"])')"
}
row ps_1p1w --mode ps --gpus 1 --steps 200 --warmup 20
row ps_1p2w --mode ps --gpus 2 --steps 200 --warmup 20
row ps_1p8w --mode ps --gpus 8 --steps 200 --warmup 20
row ps_2p8w --mode ps --gpus 8 --num_ps 2 --ps_partition_mb 4 --steps 200 --warmup 20
row ps_1p8w_b --mode ps --gpus 8 --steps 200 --warmup 20
