# Ablations of the MNIST conv kernels through rocprofv3 kernel durations (scripts/abl.sh).
set -o pipefail
O=gpurun_out/r3m
mkdir -p $O
bash scripts/abl.sh $O DTFE_C1W_DIAG "0 1 2 4 8 7 15" conv1_wgrad conv1c_wgrad || exit 1
bash scripts/abl.sh $O DTFE_C1_DIAG "0 1 2 4 8 6 7" conv1_fwd conv1c_fwd || exit 1
bash scripts/abl.sh $O DTFE_IW_DIAG "0 1 2 4 6 7" conv2_wgrad_ws imgwgrad_persist || exit 1
bash scripts/abl.sh $O DTFE_IC_DIAG "0 1 2 4 6 7" conv2_fwd,conv2_dgrad imgconv_fixed || exit 1
exit 0
