# Round-4: ps data-plane probes - Adam over an uncached vs cached gradient, 1 ps + 1 worker bench;
# fc1 GEMMs on 128x128 tiles with split-K (verdict item 4 measurement).
set -o pipefail
O=gpurun_out/r4ps
mkdir -p $O
timeout -k 10 120 python3 bench/ps_mailbox.py > $O/mailbox.txt 2>&1 || { tail -5 $O/mailbox.txt; exit 1; }
grep -v amdgpu.ids $O/mailbox.txt
timeout -k 10 240 python3 bench.py --mode ps --gpus 1 --steps 200 --warmup 20 > $O/ps11.log 2>&1 || { tail -5 $O/ps11.log; exit 1; }
grep '^{' $O/ps11.log | cut -c1-200
timeout -k 10 300 python3 bench/gemm_sweep.py --iters 30 --tiles 5,9 --splits 1,2,4,8 > $O/sweep128.txt 2>&1 || { tail -5 $O/sweep128.txt; exit 1; }
grep -v amdgpu.ids $O/sweep128.txt
