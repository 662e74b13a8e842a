#!/usr/bin/env python3
"""Per-kernel resources (VGPRs, SGPRs, spills, LDS, occupancy) from a
hipcc -save-temps .s file: tools/kres.py <file.s> [name filter]."""
import re, subprocess, sys
s = open(sys.argv[1]).read()
flt = sys.argv[2] if len(sys.argv) > 2 else ""
meta = s[s.index("amdhsa.kernels:"):]
for blk in meta.split("\n  - ")[1:]:
    g = lambda k: (re.search(r"\.%s:\s+(\S+)" % k, blk) or [None, "?"])[1]
    name = g("name")
    dn = subprocess.run(["c++filt"], input=name, capture_output=True, text=True).stdout.strip()
    if flt in dn:
        print("vgpr %s agpr %s sgpr %s vspill %s sspill %s lds %s  %s" % (
            g("vgpr_count"), g("agpr_count"), g("sgpr_count"), g("vgpr_spill_count"), g("sgpr_spill_count"),
            g("group_segment_fixed_size"), dn[:110]))
