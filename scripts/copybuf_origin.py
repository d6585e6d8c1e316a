"""Where the steady-state __amd_rocclr_copyBuffer dispatches of a kernel trace sit: for each one in the
last `--steps` steps (a step starts at `--marker`), the kernels right before and after it and its
queue.   python scripts/copybuf_origin.py <kernel_trace.csv> <marker substring> [--steps 3]"""
import argparse
import collections
import csv

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("marker")
ap.add_argument("--steps", type=int, default=3)
a = ap.parse_args()
rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if a.marker in r["Kernel_Name"]]
lo = starts[-a.steps - 1] if len(starts) > a.steps else 0
hi = starts[-1]
win = rows[lo:hi]
cp = [i for i, r in enumerate(win) if "copyBuffer" in r["Kernel_Name"]]
print("steps %d, kernels %d, copyBuffer %d (%.1f per step)" % (a.steps, len(win), len(cp), len(cp) / a.steps))
t0 = int(win[0]["Start_Timestamp"])
prev = collections.Counter()
for i in cp:
    p = next((win[j]["Kernel_Name"][:70] for j in range(i - 1, -1, -1) if "copyBuffer" not in win[j]["Kernel_Name"]), "-")
    prev[p] += 1
print("kernel preceding each copyBuffer (count):")
for k, v in prev.most_common(20):
    print("  %4d  %s" % (v, k))
print("first 12 copyBuffer dispatches in the window:")
for i in cp[:12]:
    r = win[i]
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print("  t=%9.1f us  %5.2f us  queue %s  grid %s x %s  prev=%s" % ((s - t0) / 1e3, (e - s) / 1e3, r["Queue_Id"],
          r["Grid_Size_X"], r["Workgroup_Size_X"], win[i - 1]["Kernel_Name"][:50]))
