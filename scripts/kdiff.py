"""Per-step kernel time diff: a rocprofv3 kernel_stats.csv against a profiles/ kernel table
(name / calls / slot / dur columns, as profiles/r5_resnet20_b256_kernels.txt).

    python scripts/kdiff.py <run_kernel_stats.csv> <steps in the trace> <old table.txt>"""
import csv
import re
import sys


def norm(n):
    return n.replace("(anonymous namespace)::", "").replace("void ", "").replace("dtfe::", "")[:60].strip()


steps = float(sys.argv[2])
new = {}
for r in csv.DictReader(open(sys.argv[1])):
    k = norm(r["Name"])
    c, t = new.get(k, (0, 0))
    new[k] = (c + int(r["Calls"]) / steps, t + float(r["TotalDurationNs"]) / 1e3 / steps)
old = {}
for line in open(sys.argv[3]):
    m = re.match(r"(.{62})\s+(\d+)\s+([\d.]+)\s+([\d.]+)", line)
    if m:
        old[norm(m.group(1))] = (int(m.group(2)), float(m.group(4)))
rows = []
for k in set(new) | set(old):
    n, o = new.get(k, (0, 0)), old.get(k, (0, 0))
    rows.append((n[1] - o[1], k, o, n))
for d, k, o, n in sorted(rows):
    if abs(d) > 1:
        print("%7.1f  old %4.1fx %6.1f  new %4.1fx %6.1f  %s" % (d, o[0], o[1], n[0], n[1], k))
print("total old %.1f new %.1f" % (sum(v[1] for v in old.values()), sum(v[1] for v in new.values())))
