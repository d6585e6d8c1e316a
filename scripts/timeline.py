"""One training step's kernel timeline from a rocprofv3 --kernel-trace CSV.

    python scripts/timeline.py <run_kernel_trace.csv> <first-kernel-of-step substring> [step index]

Prints start offset / duration / end (us, relative to the step's first kernel) and the
queue of every kernel of the chosen step, plus the step's wall span and the sum of the
kernel durations (their ratio is the overlap the side streams buy)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
marker = sys.argv[2]
starts = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
k = int(sys.argv[3]) if len(sys.argv) > 3 else len(starts) // 2
a, b = starts[k], starts[k + 1] if k + 1 < len(starts) else len(rows)
t0 = int(rows[a]["Start_Timestamp"])
span_end = t0
busy = 0.0
for r in rows[a:b]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    span_end = max(span_end, e)
    busy += (e - s) / 1000
    name = r["Kernel_Name"].replace("void ", "").replace("dtfe::", "").replace("(anonymous namespace)::", "")[:70]
    print("%8.1f %7.1f %8.1f  q%-3s %s" % ((s - t0) / 1000, (e - s) / 1000, (e - t0) / 1000, r.get("Queue_Id", "?"), name))
nxt = int(rows[b]["Start_Timestamp"]) if b < len(rows) else span_end
print("step span %.1f us (to next step start %.1f us), kernel sum %.1f us" % ((span_end - t0) / 1000,
                                                                            (nxt - t0) / 1000, busy))
