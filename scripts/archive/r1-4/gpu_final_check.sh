# Round-end driver paths on one GPU: smoke(), bench.py with no flags, and a 2-rank
# torchrun rehearsal of the data-parallel bench (both ranks share the one GPU; IPC comm
# over a gloo process group, since RCCL refuses two ranks on one device).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 180 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 180 python3 bench.py > gpurun_out/b_default.log 2>&1 &&
HSA_ENABLE_IPC_MODE_LEGACY=0 timeout -k 10 240 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 50 --warmup 10 \
  --comm ipc --backend gloo > gpurun_out/b_dp2_rehearsal.log 2>&1
rc=$?
tail -n 1 gpurun_out/smoke.log; tail -n 1 gpurun_out/b_default.log; grep '^{' gpurun_out/b_dp2_rehearsal.log || tail -20 gpurun_out/b_dp2_rehearsal.log
exit $rc
