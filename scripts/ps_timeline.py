"""Merged kernel timeline of a 1 ps + N worker run on one GPU (rocprofv3 --kernel-trace -o run_%pid%):
every process's kernels on one clock, labelled ps / worker, for two consecutive worker steps, plus
the median per-request ps kernel durations.

    python scripts/ps_timeline.py <dir with run_<pid>_kernel_trace.csv files> [step index]
"""
import csv
import glob
import os
import statistics
import sys

files = sorted(glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True))
rows = []
for f in files:
    rs = list(csv.DictReader(open(f)))
    names = {r["Kernel_Name"] for r in rs}
    role = "worker" if any("conv1c_fwd" in n for n in names) else "ps"
    for r in rs:
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), role, r.get("Queue_Id", "?"), r["Kernel_Name"]))
rows.sort()
wk = [r for r in rows if r[2] == "worker"]
starts = [r[0] for r in wk if "conv1c_fwd" in r[4]]
if len(starts) < 4:
    sys.exit("fewer than 4 worker steps in the trace")
k = int(sys.argv[2]) if len(sys.argv) > 2 else len(starts) // 2
t0, t1 = starts[k], starts[min(k + 2, len(starts) - 1)]
print("# two worker steps from step %d, us from its conv1 start (period %.1f us)" % (k, (starts[k + 1] - starts[k]) / 1e3))
for s, e, role, q, n in rows:
    if t0 - 30000 <= s < t1:
        print("%-6s q%-3s %-48s %+9.1f  dur %7.1f" % (role, q, n[:48], (s - t0) / 1e3, (e - s) / 1e3))
ps = [r for r in rows if r[2] == "ps"]
per = {}
for s, e, role, q, n in ps:
    per.setdefault(n.split("(")[0][:48], []).append((e - s) / 1e3)
print("# ps kernels: median duration (count)")
for n, v in sorted(per.items(), key=lambda kv: -statistics.median(kv[1])):
    print("  %-48s %7.1f us  (%d)" % (n, statistics.median(v), len(v)))
periods = [(b - a) / 1e3 for a, b in zip(starts[1:], starts[2:])]
print("# worker step period: median %.1f us over %d steps" % (statistics.median(periods), len(periods)))
