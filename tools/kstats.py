#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel_stats.csv per detection:
tools/kstats.py <csv> [detections]

The detection count defaults to the call count of k_extrema (one launch per
detection, whole-image or batched), so `per_det_us` is the kernel time one
detection spends in that kernel; `avg_us` is the kernel's own average launch
duration (what the bench's roofline events and the per-octave figures are
compared against)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
if len(sys.argv) > 2:
    dets = int(sys.argv[2])
else:
    dets = sum(int(r["Calls"]) for r in rows if r["Name"].split("(")[0].split("<")[0].endswith("k_extrema"))
    if dets == 0:
        sys.exit("no k_extrema launches: pass the detection count")
print("# detections %d (%s)" % (dets, "given" if len(sys.argv) > 2 else "k_extrema launches"))
tot = 0.0
for r in rows:
    n = r["Name"]
    if "rocprim" in n:
        short = "rocprim:" + n.split("detail::")[2][:50] if n.count("detail::") > 1 else n[:60]
    else:
        short = n.split("(")[0]
    per = float(r["TotalDurationNs"]) / 1e3 / dets
    tot += per
    print("%-70s calls/det %5.2f avg_us %9.1f per_det_us %9.1f" % (short[:70], int(r["Calls"]) / dets,
                                                                  float(r["AverageNs"]) / 1e3, per))
print("total per detection us %.1f" % tot)
