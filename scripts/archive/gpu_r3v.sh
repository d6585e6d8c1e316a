# PMC counters of the ResNet-50 implicit-GEMM convs (B=256): LDS instructions / bank conflicts vs
# MFMA busy, to decide between the 16x16x32 and 32x32x16 fragment shapes.
set -o pipefail
mkdir -p gpurun_out/r3v
bash scripts/pmc.sh r3v_convs -- python3 bench/resnet50_convs.py --batch 256 --reps 2 --no-torch > gpurun_out/r3v/pmc.txt 2>&1 || { tail -5 gpurun_out/r3v/pmc.txt; exit 1; }
grep -E "^kernel|igemm" gpurun_out/r3v/pmc.txt | cut -c1-400
