#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel_stats.csv per step: tools/kstats.py <csv> <steps>"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 1
tot = 0.0
for r in rows:
    n = r["Name"]
    if "rocprim" in n:
        short = "rocprim:" + n.split("detail::")[2][:50] if n.count("detail::") > 1 else n[:60]
    else:
        short = n.split("(")[0]
    per = float(r["TotalDurationNs"]) / 1e3 / steps
    tot += per
    print("%-70s calls/step %5.1f avg_us %9.1f per_step_us %9.1f" % (short[:70], int(r["Calls"]) / steps,
                                                                    float(r["AverageNs"]) / 1e3, per))
print("total per step us %.1f" % tot)
