set -o pipefail
mkdir -p gpurun_out
# 2-rank rehearsal of the data-parallel bench path on ONE GPU (gloo; the driver's N>1 runs use RCCL)
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 20 --warmup 3 --backend gloo --batch_size 256 > gpurun_out/b_dp2.log 2>&1; tail -3 gpurun_out/b_dp2.log
