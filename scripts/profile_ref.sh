# usage: bash scripts/profile_ref.sh <model>   -> gpurun_out/prof_ref_<model>/
set -o pipefail
m=$1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/prof_ref_$m
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ref_$m -o run -- python3 bench/ref_models.py --models $m --steps 30 --warmup 5 > gpurun_out/prof_ref_$m/stdout.log 2>&1
