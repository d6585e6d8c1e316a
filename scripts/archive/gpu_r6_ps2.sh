# Round 6: 2-ps partitioned rows at fewer ranks (is the 2 ps + 8 workers rehearsal's 55 ms a 10-process effect?)
set -o pipefail
O=gpurun_out/${1:-r6ps2}
mkdir -p $O
row() {
  local tag=$1; shift
  timeout -k 10 300 python3 bench.py "$@" > $O/$tag.log 2>&1 || { tail -5 $O/$tag.log; exit 1; }
  echo "$tag $(tail -1 $O/$tag.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d["median_window_ms_per_step"], d["window_ms_per_step"])')"
}
row ps_2p2w --mode ps --gpus 2 --num_ps 2 --ps_partition_mb 4 --steps 200 --warmup 20
row ps_1p6w --mode ps --gpus 6 --steps 200 --warmup 20
row ps_2p6w --mode ps --gpus 6 --num_ps 2 --ps_partition_mb 4 --steps 200 --warmup 20
row ps_2p7w --mode ps --gpus 7 --num_ps 2 --ps_partition_mb 4 --steps 200 --warmup 20
row ps_2p8w_nopart --mode ps --gpus 8 --num_ps 2 --steps 200 --warmup 20
