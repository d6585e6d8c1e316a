"""Per-kernel average time (us) from a rocprofv3 kernel_stats.csv, plus the per-step sum."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
import collections
steps = collections.Counter(int(r["Calls"]) for r in rows).most_common(1)[0][0]
tot = 0.0
for r in rows:
    n = r["Name"].replace("(anonymous namespace)::", "").replace("void ", "").replace("dtfe::", "")[:72]
    avg = float(r["AverageNs"]) / 1000
    calls = int(r["Calls"])
    tot += avg * calls / steps
    print(f"{avg:8.1f} us  x{calls:4d}  {n}")
print(f"per-step kernel time ~ {tot:.1f} us")
