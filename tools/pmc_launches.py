#!/usr/bin/env python3
"""Per-launch HBM bytes (and TA / L2 counters) of every kernel of one
detection, from rocprofv3 --pmc passes, grouped by (kernel, grid).

  FETCH_SIZE and WRITE_SIZE come from separate passes (TCC budget); bytes =
  2 x FETCH_SIZE x 1024 + WRITE_SIZE x 1024 (MI355X_MICROARCH.md, HBM: gfx950
  FETCH_SIZE counts half of wide streaming reads).
  The optional third pass (TA_TA_BUSY_sum TCC_HIT_sum TCC_MISS_sum
  GRBM_GUI_ACTIVE) gives the TA busy fraction (TA_TA_BUSY_sum over 256 TAs x
  GRBM_GUI_ACTIVE / 8 cycles) and the L2 hit rate.
  The optional fourth pass (SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_LDS
  SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE) gives the fp64 FMA issue
  fraction: a wave64 v_fma_f64 occupies its SIMD 4 cycles (78.6 TFLOP/s fp64
  vector peak = 1024 SIMDs x 16 lanes x 2 x 2.4 GHz), so fma_issue_frac =
  4 x SQ_INSTS_VALU_FMA_F64 / (1024 x GRBM_GUI_ACTIVE / 8); valu_issue_frac
  the same for every VALU instruction (4 cycles each, an upper estimate).

The k_gauss_dog launches of one image are ordered by grid size (octave 0 has
the largest grid); their sum is the pass's HBM traffic (`pass_hbm_bytes`),
octave 0's is `hbm_bytes_per_launch` (bench.py reads both).

The pass's traffic includes the split vertical pass (k_gauss_vert) of the
large-radius octaves.

usage: tools/pmc_launches.py --config-key KEY --out FILE FETCH_DIR WRITE_DIR [TA_DIR [SQ_DIR]]
"""
import argparse
import collections
import csv
import glob
import json
import os

N_TA = 256  # one texture addresser per CU
N_SIMD = 1024  # 256 CUs x 4 SIMDs


def collect(d):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].split("(")[0]
            if name.startswith("void "):
                name = name[5:]
            grid = int(float(r.get("Grid_Size") or r.get("Grid_Size_X") or 0))
            acc[(name, grid)][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return acc


def avg(v):
    return sum(v) / len(v) if v else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config-key", required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("ta_dir", nargs="?")
    ap.add_argument("sq_dir", nargs="?")
    a = ap.parse_args()
    F, Wr = collect(a.fetch_dir), collect(a.write_dir)
    T = collect(a.ta_dir) if a.ta_dir else {}
    Q = collect(a.sq_dir) if a.sq_dir else {}
    launches = []
    for key in sorted(set(F) | set(Wr)):
        name, grid = key
        fk = avg(F.get(key, {}).get("FETCH_SIZE", []))
        wk = avg(Wr.get(key, {}).get("WRITE_SIZE", []))
        rec = {"kernel": name, "grid": grid,
               "dispatches": [len(F.get(key, {}).get("FETCH_SIZE", [])), len(Wr.get(key, {}).get("WRITE_SIZE", []))],
               "fetch_bytes": None if fk is None else 2.0 * fk * 1024.0,
               "write_bytes": None if wk is None else wk * 1024.0}
        rec["hbm_bytes"] = (rec["fetch_bytes"] or 0.0) + (rec["write_bytes"] or 0.0)
        t = T.get(key, {})
        gui = avg(t.get("GRBM_GUI_ACTIVE", []))
        ta = avg(t.get("TA_TA_BUSY_sum", []))
        if gui and ta is not None:
            rec["ta_busy_frac"] = ta / (N_TA * gui / 8.0)
        hit, miss = avg(t.get("TCC_HIT_sum", [])), avg(t.get("TCC_MISS_sum", []))
        if hit is not None and miss is not None and hit + miss > 0:
            rec["l2_hit_rate"] = hit / (hit + miss)
        q = Q.get(key, {})
        qgui = avg(q.get("GRBM_GUI_ACTIVE", []))
        if qgui:
            cyc = N_SIMD * qgui / 8.0
            for c, k in (("SQ_INSTS_VALU_FMA_F64", "fma_issue_frac"), ("SQ_INSTS_VALU", "valu_issue_frac")):
                v = avg(q.get(c, []))
                if v is not None:
                    rec[k] = 4.0 * v / cyc
            for c in ("SQ_INSTS_VALU", "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR"):
                v = avg(q.get(c, []))
                if v is not None:
                    rec[c.lower()] = v
            rec["cycles"] = qgui / 8.0
        launches.append(rec)
    gauss = sorted([r for r in launches if "k_gauss_dog" in r["kernel"]], key=lambda r: -r["grid"])
    vert = [r for r in launches if "k_gauss_vert" in r["kernel"]]
    for o, r in enumerate(gauss):
        r["octave"] = o
    launches.sort(key=lambda r: -r["hbm_bytes"])
    out = {
        "config_key": a.config_key,
        "pass_hbm_bytes": sum(r["hbm_bytes"] for r in gauss + vert),
        "hbm_bytes_per_launch": gauss[0]["hbm_bytes"] if gauss else None,
        "kernel": "k_gauss_dog (octave 0); pass_hbm_bytes = all octaves' k_gauss_dog launches of one image "
                  "plus the split vertical pass (k_gauss_vert)",
        "launches": launches,
        "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes, averaged per "
                  "(kernel, grid) over dispatches; bytes = 2 x FETCH_SIZE x 1024 + WRITE_SIZE x 1024 "
                  "(MI355X_MICROARCH.md, HBM); TA busy = TA_TA_BUSY_sum / (256 x GRBM_GUI_ACTIVE / 8)",
    }
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    for r in launches:
        print("%-44s grid %9d  %8.1f MB read %8.1f MB written%s%s%s%s" % (
            r["kernel"][:44], r["grid"], (r["fetch_bytes"] or 0) / 1e6, (r["write_bytes"] or 0) / 1e6,
            "  TA busy %.2f" % r["ta_busy_frac"] if "ta_busy_frac" in r else "",
            "  L2 hit %.2f" % r["l2_hit_rate"] if "l2_hit_rate" in r else "",
            "  fp64 FMA issue %.2f" % r["fma_issue_frac"] if "fma_issue_frac" in r else "",
            "  VALU issue %.2f" % r["valu_issue_frac"] if "valu_issue_frac" in r else ""))
    print("pass: %.1f MB" % (out["pass_hbm_bytes"] / 1e6))


if __name__ == "__main__":
    main()
