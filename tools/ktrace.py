#!/usr/bin/env python3
"""Per-dispatch durations of the last step in a rocprofv3 kernel_trace.csv:
tools/ktrace.py <csv> [n_last]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 30
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
t0 = int(rows[-n]["Start_Timestamp"])
for r in rows[-n:]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].split("(")[0][:48]
    print("%8.1f us  +%8.1f  grid %9s wg %4s lds %6s vgpr %3s  %s" % ((e - s) / 1e3, (s - t0) / 1e3, r.get("Grid_Size_X", r.get("Grid_Size", "?")),
          r.get("Workgroup_Size_X", r.get("Workgroup_Size", "?")), r.get("LDS_Block_Size", r.get("Group_Segment_Size", "?")), r.get("VGPR_Count", r.get("Arch_VGPR_Count", "?")), name))
