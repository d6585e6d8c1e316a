"""Per-step kernel breakdown from a rocprofv3 kernel_trace.csv.

    python scripts/trace_summary.py <kernel_trace.csv> <step-marker-kernel-substring> [every]

Step boundaries are the start times of the marker kernel (one launch per step; `every`
keeps one marker in N for kernels launched several times per step).  Prints the median
step wall time, the busy (kernel) time of the middle step and its per-kernel totals."""
import collections
import csv
import statistics
import sys

path, marker = sys.argv[1], sys.argv[2]
every = int(sys.argv[3]) if len(sys.argv) > 3 else 1
rows = list(csv.DictReader(open(path)))
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
starts = [k[0] for k in ks if marker in k[2]][::every]
steps = [(b - a) / 1000 for a, b in zip(starts, starts[1:])]
mid = len(starts) // 2
a, b = starts[mid], starts[mid + 1]
agg, cnt = collections.defaultdict(float), collections.Counter()
for s, e, n in ks:
    if a <= s < b:
        n = n.replace("(anonymous namespace)::", "").replace("void ", "").replace("dtfe::", "")[:90]
        agg[n] += (e - s) / 1000
        cnt[n] += 1
print("steps %d  median step %.1f us  (middle step busy %.1f us)" % (len(steps), statistics.median(steps),
                                                                    sum(agg.values())))
for n, t in sorted(agg.items(), key=lambda x: -x[1]):
    print("  %8.1f us  x%-3d %s" % (t, cnt[n], n))
