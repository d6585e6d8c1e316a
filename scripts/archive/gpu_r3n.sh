set -o pipefail
mkdir -p gpurun_out/r3n
timeout -k 10 60 ./bench/probe/glds_probe > gpurun_out/r3n/probe.txt 2>&1; cat gpurun_out/r3n/probe.txt
bash scripts/gpu_r3l.sh && bash scripts/gpu_r3m.sh
