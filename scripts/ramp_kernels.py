"""Per-kernel mean duration early vs late in a rocprofv3 kernel trace (one row per kernel name):
which kernels carry the warm-up ramp of a fresh bench process."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
by = collections.defaultdict(list)
for r in rows:
    by[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0)
print("%-60s %6s %9s %9s %9s" % ("kernel", "calls", "first20", "mid", "last40"))
for k, v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
    if len(v) < 60:
        continue
    mid = v[len(v) // 2 - 10:len(v) // 2 + 10]
    print("%-60s %6d %9.2f %9.2f %9.2f" % (k[:60], len(v), sum(v[:20]) / 20, sum(mid) / len(mid), sum(v[-40:]) / 40))
