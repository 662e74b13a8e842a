#!/usr/bin/env python3
"""Per-octave average duration of the Gaussian+DoG launches (k_gauss_dog, k_gauss_rw, k_gauss_vert) in rocprofv3
kernel_trace.csv files (octave = the launch's tile grid, Grid_Size_X x _Y):
tools/gauss_oct.py <csv>...  (one column per file), plus k_extrema / k_refine_fast."""
import csv
import sys
from collections import defaultdict

cols = []
keys = []
for path in sys.argv[1:]:
    acc = defaultdict(list)
    for r in csv.DictReader(open(path)):
        n = r["Kernel_Name"]
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        if "k_gauss_dog" in n or "k_gauss_rw" in n or "k_gauss_vert" in n:
            k = "%s grid %sx%s" % (n.split("(")[0].split("::")[-1].split("<")[0], int(r["Grid_Size_X"]) // 256,
                                   r["Grid_Size_Y"])
        elif "k_extrema" in n or "k_refine_fast" in n or "k_emit" in n:
            k = n.split("(")[0].split("::")[-1]
        else:
            continue
        acc[k].append(d)
    cols.append(acc)
    for k in acc:
        if k not in keys:
            keys.append(k)
keys.sort()
print("%-28s" % "launch (avg us)" + "".join("%18s" % p.split("/")[-2][-16:] for p in sys.argv[1:]))
for k in keys:
    print("%-28s" % k + "".join("%18s" % ("%.1f x%d" % (sum(a[k]) / len(a[k]), len(a[k])) if a.get(k) else "-")
                                for a in cols))
