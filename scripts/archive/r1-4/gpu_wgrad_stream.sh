# ResNet-50 weight gradients on a side stream: tests, A/B bench (DTFE_WGRAD_STREAM=0/1), 2-rank rehearsal.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_resnet.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/ws_tests.log 2>&1 &&
DTFE_WGRAD_STREAM=0 timeout -k 10 200 python3 bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/ws_off.log 2>&1 &&
DTFE_WGRAD_STREAM=1 timeout -k 10 200 python3 bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/ws_on.log 2>&1 &&
DTFE_WGRAD_STREAM=0 timeout -k 10 200 python3 bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/ws_off2.log 2>&1 &&
DTFE_WGRAD_STREAM=1 timeout -k 10 200 python3 bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/ws_on2.log 2>&1 &&
HSA_ENABLE_IPC_MODE_LEGACY=0 timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29531 bench.py --model resnet50 --gpus 2 --steps 6 --warmup 2 \
  --comm ipc --backend gloo > gpurun_out/ws_dp2.log 2>&1
rc=$?
tail -n 3 gpurun_out/ws_tests.log
for f in ws_off ws_on ws_off2 ws_on2; do python3 -c "import json,sys; r=json.loads(open('gpurun_out/$f.log').read().strip().splitlines()[-1]); print('$f', r['ms_per_step'], r['median_window_ms_per_step'], r['config']['last_loss'])"; done
grep '^{' gpurun_out/ws_dp2.log || tail -20 gpurun_out/ws_dp2.log
exit $rc
