#!/usr/bin/env python3
"""Average PMC counters per (kernel, grid) over dispatches and passes:
tools/pmc_summary.py [--kernel substr] <dir>..."""
import collections
import csv
import glob
import sys

args = sys.argv[1:]
filt = None
if args and args[0] == "--kernel":
    filt, args = args[1], args[2:]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for d in args:
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].split("(")[0]
            if filt and filt not in name:
                continue
            grid = r.get("Grid_Size", r.get("Grid_Size_X", "?"))
            key = "%s grid=%s" % (name[-36:], grid)
            acc[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
for key, cs in sorted(acc.items()):
    print(key)
    for c, v in sorted(cs.items()):
        print("   %-26s n=%3d avg=%.5g" % (c, len(v), sum(v) / len(v)))
