# PMC passes over the MNIST-CNN per-kernel microbench (one counter set per rocprofv3 run)
set -o pipefail
mkdir -p gpurun_out/r2g
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_ANY" \
           "SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE SQ_INST_LEVEL_VMEM SQ_INSTS_SMEM"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d gpurun_out/r2g/pmc_$i -o run -- python3 bench/cnn_kernels.py --iters 5 > gpurun_out/r2g/pmc_$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 gpurun_out/r2g/pmc_$i.log; exit 1; }
done
python3 scripts/pmc_summary.py "gpurun_out/r2g/pmc_*/**/*counter_collection.csv" > gpurun_out/r2g/pmc_cnn_summary.csv
