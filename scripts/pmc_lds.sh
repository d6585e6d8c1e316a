# one PMC pass of LDS / MFMA counters over a short no-graph MNIST CNN bench run
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA --output-format csv -d gpurun_out/pmc_lds -o run -- python3 bench.py --steps 10 --warmup 2 --no_graph > gpurun_out/pmc_lds.log 2>&1
rc=$?
python3 scripts/pmc_summary.py "gpurun_out/pmc_lds/**/*counter_collection.csv" > gpurun_out/pmc_lds_summary.csv
exit $rc
