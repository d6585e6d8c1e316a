# Round 5: PMC passes over ResNet-20's stage-1 / stage-3 whole-image conv forward (plain launches)
set -o pipefail
bash scripts/pmc.sh r20s1 -- python3 bench/resnet20_kernels.py --no_graph --only "s1 conv2 fwd" > gpurun_out/pmc_r20s1.txt 2>&1 || { tail -20 gpurun_out/pmc_r20s1.txt; exit 1; }
grep -i "imgconv\|kernel" gpurun_out/pmc_r20s1.txt | head -5
bash scripts/pmc.sh r20s3 -- python3 bench/resnet20_kernels.py --no_graph --only "s3 conv2 fwd" > gpurun_out/pmc_r20s3.txt 2>&1 || { tail -20 gpurun_out/pmc_r20s3.txt; exit 1; }
grep -i "imgconv\|kernel" gpurun_out/pmc_r20s3.txt | head -5
