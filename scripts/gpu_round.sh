set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 bench/imgconv_scan.py > gpurun_out/scan.log 2>&1; cat gpurun_out/scan.log
