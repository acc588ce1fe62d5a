"""Reads a rocprofv3 kernel_trace.csv of bench.py and prints the decision-step timeline:
for the last steps, each kernel's start/end relative to the step's first K1 start, and
the gap between consecutive steps."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
ev = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].replace("void ", "")[:28],
              r["Queue_Id"]) for r in rows), key=lambda e: e[0])
k1 = [e for e in ev if "k_pod_reduce" in e[2]]
steps = k1[-12:-1]
for i, s in enumerate(steps[:-1]):
    t0 = s[0]
    nxt = steps[i + 1][0]
    inner = [e for e in ev if t0 <= e[0] < nxt]
    print("step %d: period %.1f us" % (i, (nxt - t0) / 1e3))
    for e in inner:
        print("   q%s %-28s %7.1f -> %7.1f (%5.1f)" % (e[3], e[2], (e[0] - t0) / 1e3, (e[1] - t0) / 1e3, (e[1] - e[0]) / 1e3))
