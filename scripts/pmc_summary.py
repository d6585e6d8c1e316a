"""Summarise rocprofv3 --pmc CSV output: mean counter value per kernel (short names)."""
import collections
import csv
import glob
import re
import sys


def short(name):
    n = name.replace("(anonymous namespace)::", "")
    n = re.sub(r"\(dtfe::.*$", "", n)
    n = re.sub(r"\(.*$", "", n)
    n = n.replace("void ", "").replace("dtfe::", "")
    return n[:80]


def main(paths):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for p in paths:
        for f in glob.glob(p, recursive=True):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    k = short(row.get("Kernel_Name", ""))
                    c = row.get("Counter_Name")
                    v = row.get("Counter_Value")
                    if c and v:
                        acc[k][c].append(float(v))
    counters = sorted({c for d in acc.values() for c in d})
    w = csv.writer(sys.stdout)  # kernel names hold commas (template arguments): quote them
    w.writerow(["kernel"] + counters)
    for k, d in sorted(acc.items()):
        w.writerow([k] + [("%.4g" % (sum(d[c]) / len(d[c]))) if d.get(c) else "" for c in counters])


if __name__ == "__main__":
    main(sys.argv[1:] or ["gpurun_out/pmc*/**/*counter_collection.csv"])
