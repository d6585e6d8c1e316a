# usage: bash scripts/pmc.sh <tag> -- <python script + args>   (counter passes over one workload)
set -o pipefail
tag=$1; shift; shift
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_WR"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmc_${tag}_$i -o run -- "$@" > gpurun_out/pmc_${tag}_$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 gpurun_out/pmc_${tag}_$i.log; exit 1; }
done
python3 scripts/pmc_summary.py "gpurun_out/pmc_${tag}_*/**/*counter_collection.csv" > gpurun_out/pmc_${tag}_summary.csv
cat gpurun_out/pmc_${tag}_summary.csv
