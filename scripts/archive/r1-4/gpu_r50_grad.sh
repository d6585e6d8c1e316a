# ResNet-50 numerics on the GPU: gradient check against fp32 autograd (oracle with bf16 forward
# rounding) and the loss trajectory next to an fp32 model from the same weights and batches.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 240 python3 scripts/r50_grad_check.py --batch 256 --round > gpurun_out/r50_grad_b256_round.log 2>&1 &&
timeout -k 10 300 python3 scripts/r50_train_compare.py --batch 256 --steps 30 > gpurun_out/r50_train_cmp.log 2>&1
rc=$?
head -n 30 gpurun_out/r50_grad_b256_round.log; tail -n 1 gpurun_out/r50_grad_b256_round.log; cat gpurun_out/r50_train_cmp.log | tail -32
exit $rc
