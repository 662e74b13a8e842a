#!/usr/bin/env python3
"""Kernels of the last cfg-5 repetition's tail phase and merge, from a
rocprofv3 --kernel-trace CSV: the kernels between the last k_extrema launch
group of the bands and the last k_merge_blocks, with the idle gap before each.
usage: tail_gaps.py <kernel_trace.csv> [n_last]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n_last = int(sys.argv[2]) if len(sys.argv) > 2 else 70
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
last_merge = max(i for i, r in enumerate(rows) if "k_merge_blocks" in r["Kernel_Name"])
sel = rows[max(0, last_merge - n_last):last_merge + 2]
prev_end = None
for r in sel:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = 0.0 if prev_end is None else max(0, s - prev_end) / 1e3
    prev_end = max(prev_end or 0, e)
    print("gap %7.1f us  dur %7.1f us  %-60.60s grid %s" % (gap, (e - s) / 1e3, r["Kernel_Name"], r.get("Grid_Size", r.get("Grid_Size_X", ""))))
