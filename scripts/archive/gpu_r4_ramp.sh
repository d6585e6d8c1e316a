# clock-ramp check: the driver's shape (--steps 20 --warmup 5) vs longer untimed warmups
set -e
for w in 5 100 1000 5; do
  timeout -k 10 120 python bench.py --steps 20 --warmup $w | sed "s/^/warmup=$w /" >> gpurun_out/ramp.log
done
