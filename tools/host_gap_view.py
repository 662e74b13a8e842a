#!/usr/bin/env python3
"""Interleave the last N HIP API calls and kernels of a rocprofv3 csv trace
(--hip-trace --kernel-trace) by time: where the host is behind the GPU.
usage: tools/host_gap_view.py <dir with run_hip_api_trace.csv, run_kernel_trace.csv> [N]"""
import csv
import os
import sys

d = sys.argv[1]
N = int(sys.argv[2]) if len(sys.argv) > 2 else 120


def rows(name):
    with open(os.path.join(d, name)) as f:
        return list(csv.DictReader(f))


api = rows("run_hip_api_trace.csv")
ker = rows("run_kernel_trace.csv")
ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "api", r["Function"]) for r in api]
ev += [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "GPU", r["Kernel_Name"][:60]) for r in ker]
ev.sort()
ev = ev[-N:]
t0 = ev[0][0]
for s, e, k, n in ev:
    print("%9.1f us  %7.1f us  %-3s %s" % ((s - t0) / 1e3, (e - s) / 1e3, k, n))
