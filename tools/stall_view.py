#!/usr/bin/env python3
"""Per-kernel stall / issue view of rocprofv3 --pmc passes (gpurun_out/stall_<tag>_*):
tools/stall_view.py <tag> [kernel substring ...].  SQ wave counters are in quad-cycles."""
import collections, csv, glob, sys
tag = sys.argv[1]
flt = sys.argv[2:] or ["gauss", "extrema", "refine_fast"]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob("gpurun_out/stall_%s_*/**/*counter_collection.csv" % tag, recursive=True):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].split("(")[0]
        if not any(s in name for s in flt):
            continue
        key = (name.replace("void ", "").replace("sift::", "")[-40:], r["Grid_Size"], r["VGPR_Count"], r["LDS_Block_Size"])
        acc[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in sorted(acc.items()):
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    W = m.get("SQ_WAVES", 1); cyc = m.get("GRBM_GUI_ACTIVE", 0) / 8
    print("%s grid=%s vgpr=%s lds=%s" % k)
    g = lambda c: m.get(c, 0) / W
    print("  per wave (qc): life %.0f active %.0f wait %.0f wait_inst %.0f | valu %.0f sca %.0f lds %.0f vmem %.0f" % tuple(
        g(c) for c in ["SQ_WAVE_CYCLES", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_VALU",
                       "SQ_ACTIVE_INST_SCA", "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_VMEM"]))
    print("  per wave insts: valu %.0f fma64 %.0f salu %.0f smem %.0f lds %.0f vmrd %.0f vmwr %.0f br %.0f" % tuple(
        g(c) for c in ["SQ_INSTS_VALU", "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_SALU", "SQ_INSTS_SMEM", "SQ_INSTS_LDS",
                       "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_INSTS_BRANCH"]))
    if cyc:
        print("  kernel %.0f cyc/XCD, waves %.0f, avg waves/SIMD %.2f, VALU share %.2f, fma64 share %.2f, TA busy %.2f, TCP pend %.2f, TCC hit %.2f, LDS confl %.2f" % (
            cyc, W, m.get("SQ_WAVE_CYCLES", 0) * 4 / (cyc * 1024), m.get("SQ_ACTIVE_INST_VALU", 0) * 4 / (cyc * 1024),
            4 * m.get("SQ_INSTS_VALU_FMA_F64", 0) / (cyc * 1024), m.get("TA_TA_BUSY_sum", 0) / (cyc * 256),
            m.get("TCP_PENDING_STALL_CYCLES_sum", 0) / (cyc * 256),
            m.get("TCC_HIT_sum", 0) / max(1, m.get("TCC_HIT_sum", 0) + m.get("TCC_MISS_sum", 0)),
            m.get("SQ_LDS_BANK_CONFLICT", 0) / max(1, m.get("SQ_ACTIVE_INST_LDS", 1))))
