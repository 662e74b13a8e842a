#!/usr/bin/env python3
"""Per-kernel stall / issue summary of tools/gpu_stall_pmc.sh passes:
tools/stall_summary.py <tag> [kernel filter].  SQ wave counters are in
quad-cycles; per-wave figures = counter / SQ_WAVES; per-SIMD issue shares =
instructions x 4 cycles / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs)."""
import collections, csv, glob, sys
tag = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob("gpurun_out/stall_%s_*/**/*counter_collection.csv" % tag, recursive=True):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].split("(")[0]
        if flt not in name:
            continue
        key = "%s grid=%s" % (name[-40:], r.get("Grid_Size", r.get("Grid_Size_X", "?")))
        acc[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
for key, cs in sorted(acc.items()):
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    W = m.get("SQ_WAVES", 1)
    cyc = m.get("GRBM_GUI_ACTIVE", 0) / 8
    print(key)
    print("   per wave (quad-cycles): life %.0f, busy-VALU %.0f, wait(mem) %.0f, wait-inst %.0f, active-any %.0f, active-LDS %.0f" % (
        m.get("SQ_WAVE_CYCLES", 0) / W, m.get("SQ_ACTIVE_INST_VALU", 0) / W, m.get("SQ_WAIT_ANY", 0) / W,
        m.get("SQ_WAIT_INST_ANY", 0) / W, m.get("SQ_ACTIVE_INST_ANY", 0) / W, m.get("SQ_ACTIVE_INST_LDS", 0) / W))
    if cyc:
        per_simd = lambda n: 4 * n / (cyc * 1024)
        print("   per-SIMD issue share: VALU %.2f (fp64 fma %.2f), LDS instr/SIMD-cycle %.3f, SALU %.2f; LDS bank-conflict cycles / LDS active %.2f; waves %.0f" % (
            per_simd(m.get("SQ_INSTS_VALU", 0)), per_simd(m.get("SQ_INSTS_VALU_FMA_F64", 0)),
            m.get("SQ_INSTS_LDS", 0) / (cyc * 1024), m.get("SQ_INSTS_SALU", 0) / (cyc * 1024),
            m.get("SQ_LDS_BANK_CONFLICT", 0) / max(1, m.get("SQ_ACTIVE_INST_LDS", 1)), W))
        print("   TA busy %.2f, TCP pending stall %.2f, TCC hit %.2f; GRBM cycles %.0f" % (
            m.get("TA_TA_BUSY_sum", 0) / (cyc * 256), m.get("TCP_PENDING_STALL_CYCLES_sum", 0) / (cyc * 256),
            m.get("TCC_HIT_sum", 0) / max(1, m.get("TCC_HIT_sum", 0) + m.get("TCC_MISS_sum", 0)), cyc))
