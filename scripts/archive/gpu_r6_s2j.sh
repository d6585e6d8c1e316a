# Round 6 (session 2): isolated times + PMC of the MNIST conv2 kernels (fwd, dgrad, wgrad with its workspace)
set -o pipefail
O=gpurun_out/${1:-r6s2j}
mkdir -p $O
timeout -k 10 200 python3 bench/cnn_kernels.py --iters 50 > $O/kern.log 2>&1 || { tail -5 $O/kern.log; exit 1; }
grep -v amdgpu.ids $O/kern.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for op in conv2_fwd conv2_dgrad conv2_wgrad_ws conv1_wgrad; do
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_SMEM" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC" \
           "SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE SQ_INST_LEVEL_VMEM SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_ANY"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d $O/${op}_$i -o run -- python3 bench/cnn_kernels.py --only $op --iters 2 > $O/${op}_$i.log 2>&1 || { echo "pmc pass $op $i failed"; tail -5 $O/${op}_$i.log; exit 1; }
done
python3 scripts/pmc_summary.py "$O/${op}_*/**/*counter_collection.csv" | grep -v "at::native" > $O/${op}_summary.csv
cat $O/${op}_summary.csv
done
