# CNN fc1-wgrad Adam epilogue + PS bucket applies + stem BN partials + tapless dgrad phases:
# GPU tests, CNN A/B (alternating, driver-shaped bench), ResNet-50 bench, CNN rocprof, ResNet-50
# bf16-vs-AMP gradient table.
set -o pipefail
O=gpurun_out/r3b
mkdir -p $O
timeout -k 10 800 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_mnist_cnn_gpu.py tests/test_resnet.py tests/test_norm_gpu.py tests/test_kernels_gpu.py tests/test_igemm_tiles_gpu.py tests/test_cluster_gpu.py > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -20; exit $rc; }
b() { tag=$1; shift; timeout -k 10 200 env "$@" python3 bench.py --steps 200 --warmup 20 > $O/b_$tag.log 2>&1 && echo "$tag $(grep '^{' $O/b_$tag.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["median_window_ms_per_step"], d["config"]["last_loss"])')"; }
for rep in 1 2 3; do b fused$rep DTFE_CNN_FUSED_ADAM=1 && b sep$rep DTFE_CNN_FUSED_ADAM=0 || exit 1; done
timeout -k 10 300 python3 bench.py --model resnet50 --steps 20 --warmup 5 > $O/r50.log 2>&1 || exit 1
tail -1 $O/r50.log | cut -c1-220
timeout -k 10 200 python3 bench.py --mode ps --gpus 1 --steps 200 --warmup 20 > $O/ps1.log 2>&1 || exit 1
tail -1 $O/ps1.log | cut -c1-260
timeout -k 10 300 python3 scripts/r50_grad_check.py --amp --batch 64 > $O/r50_amp.txt 2>&1 || exit 1
tail -3 $O/r50_amp.txt
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_cnn -o run -- python3 bench.py --steps 30 --warmup 5 > $O/prof_cnn.log 2>&1 || exit 1
f=$(find $O/prof_cnn -name "*kernel_stats.csv" | head -1); python3 scripts/kstats.py "$f" > $O/cnn_kernels.txt; head -16 $O/cnn_kernels.txt
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_r50 -o run -- python3 bench.py --model resnet50 --steps 8 --warmup 5 > $O/prof_r50.log 2>&1 || exit 1
f=$(find $O/prof_r50 -name "*kernel_stats.csv" | head -1); python3 scripts/kstats.py "$f" > $O/r50_kernels.txt; head -30 $O/r50_kernels.txt
