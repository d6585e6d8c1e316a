set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 bench/resnet50_convs.py --reps 10 > gpurun_out/r50_convs.log 2>&1
rc=$?
cat gpurun_out/r50_convs.log
exit $rc
