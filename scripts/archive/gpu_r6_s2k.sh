# Round 6 (session 2): conv2 weight-gradient grid below 160 (fewer partial slabs for the reduce)
set -o pipefail
O=gpurun_out/${1:-r6s2k}
mkdir -p $O
timeout -k 10 500 python3 bench/cnn_ab.py --arms "c2_blocks=192" "c2_blocks=96" "c2_blocks=128" "c2_blocks=144" --rounds 2 > $O/ab.log 2>&1 || { tail -5 $O/ab.log; exit 1; }
grep ms/step $O/ab.log
