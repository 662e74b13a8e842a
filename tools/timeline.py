#!/usr/bin/env python3
"""Concurrency profile of a pipelined bench run from a rocprofv3 kernel trace:
over the steady-state window (middle 80 % of the run), the fraction of wall
time each kernel class is running, how many kernels overlap, and the wall
time per image.  usage: tools/timeline.py run_kernel_trace.csv"""
import collections
import csv
import sys


def klass(name, grid):
    if "k_gauss_dog<true" in name:
        return "gauss o0"
    if "k_gauss_dog" in name:
        return "gauss o>=1"
    for k in ("k_extrema", "k_refine_fast", "k_refine_exact", "k_emit", "k_exact_extrema"):
        if k in name:
            return k
    return "other"


rows = list(csv.DictReader(open(sys.argv[1])))
ev = []
for r in rows:
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), klass(r["Kernel_Name"], r.get("Grid_Size"))))
ev.sort()
t0, t1 = ev[0][0], max(e[1] for e in ev)
w0, w1 = t0 + (t1 - t0) // 10, t1 - (t1 - t0) // 10
# sweep
pts = []
for s, e, k in ev:
    s, e = max(s, w0), min(e, w1)
    if e > s:
        pts.append((s, 1, k))
        pts.append((e, -1, k))
pts.sort()
active = collections.Counter()
busy = collections.Counter()      # time class k is active
alone = collections.Counter()     # time class k is the only class active
conc = collections.Counter()      # time with n kernels active
last = w0
for t, d, k in pts:
    dt = t - last
    if dt > 0:
        n = sum(active.values())
        conc[n] += dt
        for c, v in active.items():
            if v:
                busy[c] += dt
        live = [c for c, v in active.items() if v]
        if len(live) == 1:
            alone[live[0]] += dt
    active[k] += d
    last = t
W = w1 - w0
n_img = sum(1 for s, e, k in ev if k == "gauss o0" and w0 <= s < w1)
print("window %.2f ms, %d images -> %.4f ms per image" % (W / 1e6, n_img, W / 1e6 / max(n_img, 1)))
for c in sorted(busy, key=lambda c: -busy[c]):
    print("  %-16s busy %5.1f %%  alone %5.1f %%  (%.4f ms per image)" % (c, 100 * busy[c] / W, 100 * alone[c] / W,
                                                                          busy[c] / 1e6 / max(n_img, 1)))
print("  kernels running: " + ", ".join("%d: %.1f %%" % (n, 100 * v / W) for n, v in sorted(conc.items())))
