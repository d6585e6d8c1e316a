# Kernel ablation through rocprofv3 kernel durations (not host-bound event timing):
#   bash scripts/abl.sh <outdir> <ENV_NAME> "<values>" <cnn_kernels ops> <kernel-name substring>
# runs bench/cnn_kernels.py --only <ops> once per ENV_NAME value and prints the kernel's mean duration.
set -o pipefail
O=$1; VAR=$2; VALS=$3; OPS=$4; KN=$5
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for v in $VALS; do
  ( export $VAR=$v; timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/abl_${VAR}_$v -o run -- python3 bench/cnn_kernels.py --iters 5 --only $OPS > $O/abl_${VAR}_$v.log 2>&1 ) || { echo "ablation $VAR=$v failed"; tail -3 $O/abl_${VAR}_$v.log; exit 1; }
  f=$(find $O/abl_${VAR}_$v -name "*kernel_stats.csv" | head -1)
  echo "$VAR=$v $(python3 -c "
import csv,sys
for r in csv.DictReader(open('$f')):
    if '$KN' in r['Name']: print('%s avg %.1f us min %.1f us calls %s' % (r['Name'][:40], float(r['AverageNs'])/1e3, float(r['MinNs'])/1e3, r['Calls']))
")"
done
