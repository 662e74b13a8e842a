#!/usr/bin/env python3
"""Average duration per kernel name in rocprofv3 kernel_trace.csv files:
tools/ktavg.py <csv>...  (one column per file)"""
import csv
import sys
from collections import defaultdict

cols = []
names = []
for path in sys.argv[1:]:
    acc = defaultdict(list)
    for r in csv.DictReader(open(path)):
        n = r["Kernel_Name"].split("(")[0]
        if "rocprim" in n:
            n = "rocprim:" + n.split("::")[-1][:30]
        acc[n[:44]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    cols.append(acc)
    for n in acc:
        if n not in names:
            names.append(n)
print("%-46s" % "kernel (avg us, calls)" + "".join("%22s" % p.split("/")[-2][:20] for p in sys.argv[1:]))
for n in names:
    row = "%-46s" % n
    for acc in cols:
        v = acc.get(n)
        row += "%22s" % ("%.1f x%d" % (sum(v) / len(v), len(v)) if v else "-")
    print(row)
