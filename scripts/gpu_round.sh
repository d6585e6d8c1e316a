set -o pipefail
mkdir -p gpurun_out
DTFE_IC_WAVES=16 timeout -k 10 600 python3 -m pytest tests/test_imgconv.py -x -q -k persist > gpurun_out/t_k.log 2>&1; echo "TEST EXIT $?" >> gpurun_out/t_k.log
tail -2 gpurun_out/t_k.log
grep -q "TEST EXIT 0" gpurun_out/t_k.log || { grep -E "assert|Error|FAIL" gpurun_out/t_k.log | head -20; exit 1; }
DTFE_IC_WAVES=16 timeout -k 10 300 python3 bench/imgconv_scan.py > gpurun_out/scan16.log 2>&1; cat gpurun_out/scan16.log
