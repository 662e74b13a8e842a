#!/usr/bin/env python3
"""Average PMC counters per kernel name over the passes: tools/pmc_summary.py <dir>..."""
import collections
import csv
import glob
import sys

acc = collections.defaultdict(lambda: collections.defaultdict(list))
for d in sys.argv[1:]:
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].split("(")[0][-40:]
            acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
for name, cs in sorted(acc.items()):
    print(name)
    for c, v in sorted(cs.items()):
        print("   %-28s n=%3d avg=%.4g" % (c, len(v), sum(v) / len(v)))
