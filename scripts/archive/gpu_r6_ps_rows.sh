#!/bin/bash
# Round 6: the 9- / 10-rank one-GPU PS rehearsals at 200 timed steps (50 steps let one start-up stall dominate).
set -o pipefail
O=gpurun_out/r6psr; mkdir -p $O
for tag in ps_1p8w ps_2p8w; do
  args="--mode ps --gpus 8 --steps 200 --warmup 20"; [ $tag = ps_2p8w ] && args="$args --num_ps 2 --ps_partition_mb 4"
  timeout -k 10 300 python3 bench.py $args > $O/$tag.log 2>&1 || { tail -5 $O/$tag.log; exit 1; }
  echo "$tag $(tail -1 $O/$tag.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d.get("window_ms_per_step"))')"
done
