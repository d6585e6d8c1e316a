# HIP graph runtime knobs vs the CNN step (A/B, one GPU): how many hardware queues the graph's
# parallel branches are spread over decides how many cross-queue dependency edges the step pays.
set -o pipefail
O=gpurun_out/r2h
mkdir -p $O
b() { tag=$(echo "$*" | tr ' =' '_-'); timeout -k 10 180 env "$@" python3 bench.py --steps 300 --warmup 30 > $O/b_$tag.log 2>&1 && echo "$* $(grep '^{' $O/b_$tag.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["median_window_ms_per_step"])')"; }
r() { tag=$(echo "$*" | tr ' =' '_-'); timeout -k 10 180 env "$@" python3 bench/ref_models.py --steps 300 --warmup 30 > $O/r_$tag.log 2>&1 && echo "$*" && grep '^{' $O/r_$tag.log | cut -c1-80; }
b DTFE_X=base && b DEBUG_HIP_FORCE_GRAPH_QUEUES=1 && b DEBUG_HIP_FORCE_GRAPH_QUEUES=2 && b DEBUG_HIP_FORCE_GRAPH_QUEUES=3 && \
b DEBUG_HIP_FORCE_GRAPH_QUEUES=8 && b DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 && b DEBUG_HIP_GRAPH_BATCH_SIZE=1 && \
b DEBUG_HIP_GRAPH_BATCH_SIZE=64 && b DEBUG_HIP_FORCE_GRAPH_QUEUES=2 DTFE_CNN_ORDER=crit && b DEBUG_HIP_FORCE_GRAPH_QUEUES=1 DTFE_CNN_BRANCHES=none || exit 1
r DTFE_X=base && r DEBUG_HIP_FORCE_GRAPH_QUEUES=1 && r DEBUG_HIP_FORCE_GRAPH_QUEUES=2 || exit 1
exit 0
