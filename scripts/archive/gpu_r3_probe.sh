# Round-3 first look: driver-shaped bench + the multi-rank rehearsals (ranks share the one GPU via
# gloo + the hipIpc engine).  A plain failure (rc 1) moves on; a fault / abort / timeout stops.
set -o pipefail
O=gpurun_out/r3probe
mkdir -p $O
run() {  # run <tag> <timeout> <cmd...>
  tag=$1; to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$tag.log 2>&1
  rc=$?
  echo "[$tag rc=$rc] $(grep '^{' $O/$tag.log | tail -1 | cut -c1-600)"
  case $rc in 0|1|2) ;; *) tail -20 $O/$tag.log; exit $rc ;; esac
}
run n1 180 python3 bench.py --steps 20 --warmup 5
run r50w2 400 python3 bench.py --model resnet50 --gpus 2 --backend gloo --comm ipc --batch_size 32 --steps 6 --warmup 3
run cnnw8 400 python3 bench.py --gpus 8 --backend gloo --comm ipc --batch_size 256 --steps 6 --warmup 3
run r20w8 400 python3 bench.py --model resnet20 --gpus 8 --backend gloo --comm ipc --batch_size 64 --steps 4 --warmup 3
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_cluster_gpu.py > $O/cluster.log 2>&1
rc=$?; tail -3 $O/cluster.log; grep -E "PASS|FAIL" $O/cluster.log | head -20
exit $rc
