set -o pipefail
O=gpurun_out/${1:-r2k}
mkdir -p $O
for cfg in "branch fc,c2" "crit fc,c2" "branch side1" "crit side1" "branch none"; do
  set -- $cfg
  DTFE_CNN_ORDER=$1 DTFE_CNN_BRANCHES=$2 timeout -k 10 120 python3 bench.py --steps 300 --warmup 30 > $O/b_$1_$2.log 2>&1 || exit 1
  echo "$1 $2 $(grep '^{' $O/b_$1_$2.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["median_window_ms_per_step"])')"
done
