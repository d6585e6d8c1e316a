set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python3 -m pytest tests/test_resnet.py tests/test_cluster_gpu.py -q -k "conv_ops or cluster or resnet20" > gpurun_out/t_k.log 2>&1; echo "TEST EXIT $?" >> gpurun_out/t_k.log
tail -3 gpurun_out/t_k.log
grep -q "TEST EXIT 0" gpurun_out/t_k.log || { grep -E "^E  .*(Error|assert)|FAIL" gpurun_out/t_k.log | head -30; exit 1; }
