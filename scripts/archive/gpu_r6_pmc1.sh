# Round 6: PMC passes over the fc1 gradient GEMMs, tile 12 (64x64, 4 waves, ~3 WGs/CU) vs tile 22
# (256x128, 8 waves, 1 WG/CU)
set -o pipefail
O=gpurun_out/${1:-r6pmc1}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for tile in 12 22; do
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_WR" \
           "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d $O/t${tile}_$i -o run -- python3 bench/fc_probe.py --tile $tile --reps 10 > $O/t${tile}_$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $O/t${tile}_$i.log; exit 1; }
done
python3 scripts/pmc_summary.py "$O/t${tile}_*/**/*counter_collection.csv" > $O/t${tile}_summary.csv
cat $O/t${tile}_summary.csv
done
