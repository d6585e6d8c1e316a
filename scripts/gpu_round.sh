set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python3 -m pytest tests/test_resnet.py -x -q > gpurun_out/t_k.log 2>&1; echo "TEST EXIT $?" >> gpurun_out/t_k.log
tail -3 gpurun_out/t_k.log
grep -q "TEST EXIT 0" gpurun_out/t_k.log || { grep -E "^E  .*(Error|assert)|FAIL" gpurun_out/t_k.log | head -30; exit 1; }
timeout -k 10 300 python3 bench.py --model resnet20 --steps 30 --warmup 5 > gpurun_out/b_r20.log 2>&1; tail -1 gpurun_out/b_r20.log
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r20 -o run -- python3 bench.py --model resnet20 --steps 10 --warmup 3 > gpurun_out/prof_r20.log 2>&1; python3 scripts/kstats.py gpurun_out/prof_r20/run_kernel_stats.csv > gpurun_out/prof_r20.txt; head -24 gpurun_out/prof_r20.txt
