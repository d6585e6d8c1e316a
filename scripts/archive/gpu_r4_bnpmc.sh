# Round-4: BN kernel bandwidth per ResNet-50 shape at B=256; implicit-GEMM PMC (LDS conflicts, MFMA busy)
set -o pipefail
O=gpurun_out/r4bnpmc
mkdir -p $O
timeout -k 10 200 python3 bench/bn_bench.py --batch 256 > $O/bn_bench.txt 2>&1 || { tail -5 $O/bn_bench.txt; exit 1; }
grep -v amdgpu.ids $O/bn_bench.txt
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES \
  --output-format csv -d $O/pmc -o run -- python3 bench/resnet50_convs.py --batch 256 --reps 3 --no-torch --only "14,256,256,3,1;56,64,256,1,1" > $O/pmc.log 2>&1 || { tail -5 $O/pmc.log; exit 1; }
python3 scripts/pmc_summary.py "$O/pmc/**/*counter_collection.csv" > $O/pmc_summary.csv 2>&1; grep -v "at::native\|rocclr" $O/pmc_summary.csv | head -20
