#!/usr/bin/env python3
"""Per-launch HBM bytes (and TA / L2 / instruction counters) of every kernel
of one detection, from rocprofv3 --pmc passes, and the Gaussian+DoG pass's
traffic per octave.

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
  4 x SQ_INSTS_VALU_FMA_F64 / (1024 x GRBM_GUI_ACTIVE / 8).

Pass segmentation (round 5).  Every dispatch of a PMC run is serialised, and
a detection enqueues its Gaussian+DoG pass as one run of consecutive pass
launches on its queue (PASS_PREFIXES: every k_gauss_* launch, the seed-only
chain, the materialised octave-0 base) before its first non-pass kernel.
Within one detection the octaves are launched in order, so the pass's tile
launches get octaves 0, 1, 2, ... in dispatch order (a launch listed in
SPAN covers several octaves), and the helper launches (split vertical pass,
seed-only chain) are charged to the octave of the next tile launch.  Each
octave is labelled with its plane size from the configuration key.  Per
octave and over the whole pass the bytes are averaged over the detections
of each run, then FETCH (one run) and WRITE (another run) are added:
`pass_hbm_bytes` is the sum of every pass launch of one image, and
`per_octave[o].hbm_bytes` its split.

usage: tools/pmc_launches.py --config-key KEY --out FILE FETCH_DIR WRITE_DIR [TA_DIR [SQ_DIR]]
"""
import argparse
import collections
import csv
import glob
import json
import os
import re
import time

N_TA = 256  # one texture addresser per CU
N_SIMD = 1024  # 256 CUs x 4 SIMDs

PASS_PREFIXES = ("sift::k_gauss_", "sift::k_seed_", "sift::k_upsample_base")
# helper launches of the pass: charged to the octave of the next tile launch
AUX = ("sift::k_gauss_vert", "sift::k_seed_vert", "sift::k_seed_horz", "sift::k_upsample_base",
       "sift::k_gauss_seedchain")
# tile launches that cover more than one octave (name prefix -> octaves)
SPAN = {"sift::k_gauss_oct23": 2}


def kname(raw):
    name = raw.split("(")[0]
    if name.startswith("void "):
        name = name[5:]
    return name.split("<")[0]


def is_pass(name):
    return name.startswith(PASS_PREFIXES)


def dispatches(d):
    """{dispatch id: {"name", "full", "grid", "queue", counters...}} of one run."""
    out = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            did = (f, int(r["Dispatch_Id"]))
            rec = out.get(did)
            if rec is None:
                full = r["Kernel_Name"].split("(")[0]
                full = full[5:] if full.startswith("void ") else full
                rec = out[did] = {"name": kname(r["Kernel_Name"]), "full": full,
                                  "grid": int(float(r.get("Grid_Size") or r.get("Grid_Size_X") or 0)),
                                  "queue": r.get("Queue_Id"), "ctr": {}}
            rec["ctr"][r["Counter_Name"]] = rec["ctr"].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return out


def pass_segments(D):
    """Lists of the pass launches of each detection, in dispatch order."""
    byq = collections.defaultdict(list)
    for did in sorted(D, key=lambda k: (k[0], k[1])):
        byq[(did[0], D[did]["queue"])].append(D[did])
    segs = []
    for q, recs in byq.items():
        cur = []
        for rec in recs:
            if is_pass(rec["name"]):
                cur.append(rec)
            elif cur:
                segs.append(cur)
                cur = []
        if cur:
            segs.append(cur)
    return segs


def label_octaves(seg):
    """[(octave tuple, rec)] for one detection's pass launches."""
    out, pending, o = [], [], 0
    for rec in seg:
        if rec["name"].startswith(AUX):
            pending.append(rec)
            continue
        span = next((n for p, n in SPAN.items() if rec["name"].startswith(p)), 1)
        octs = tuple(range(o, o + span))
        for p in pending:
            out.append((octs, p))
        pending = []
        out.append((octs, rec))
        o += span
    for p in pending:  # trailing helpers (none in a complete pass)
        out.append(((o,), p))
    return out


def per_octave(D, counter, scale):
    """{octave tuple: mean bytes per detection}, mean pass bytes, detections."""
    segs = [s for s in pass_segments(D) if s]
    if not segs:
        return {}, None, 0
    acc = collections.defaultdict(float)
    total = 0.0
    for seg in segs:
        for octs, rec in label_octaves(seg):
            v = rec["ctr"].get(counter)
            if v is None:
                continue
            acc[octs] += v * scale
            total += v * scale
    n = len(segs)
    return {k: v / n for k, v in acc.items()}, total / n, n


def collect(d):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for rec in dispatches(d).values():
        for c, v in rec["ctr"].items():
            acc[(rec["full"], rec["grid"])][c].append(v)
    return acc


def avg(v):
    return sum(v) / len(v) if v else None


def geometry(cfg_key):
    m = re.match(r"(\d+)x(\d+)_o(\d+)_s(\d+)", cfg_key)
    if not m:
        return None
    W, H, O, S = (int(g) for g in m.groups())
    h, w, dims = 2 * H, 2 * W, []
    for o in range(O):
        if o:
            h, w = (h + 1) // 2, (w + 1) // 2
        dims.append((h, w))
    return W, H, O, S, dims


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config-key", required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--round", default=None, help="profile tag recorded in the summary (e.g. r5c)")
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("ta_dir", nargs="?")
    ap.add_argument("sq_dir", nargs="?")
    a = ap.parse_args()
    DF, DW = dispatches(a.fetch_dir), dispatches(a.write_dir)
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
            v = avg(q.get("SQ_INSTS_VALU_FMA_F64", []))
            if v is not None:
                rec["fma_issue_frac"] = 4.0 * v / cyc
            for c in ("SQ_INSTS_VALU", "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR"):
                v = avg(q.get(c, []))
                if v is not None:
                    rec[c.lower()] = v
            rec["cycles"] = qgui / 8.0
        launches.append(rec)
    launches.sort(key=lambda r: -r["hbm_bytes"])

    fo, ftot, nf = per_octave(DF, "FETCH_SIZE", 2.0 * 1024.0)
    wo, wtot, nw = per_octave(DW, "WRITE_SIZE", 1024.0)
    geo = geometry(a.config_key)
    octs = sorted(set(fo) | set(wo))
    po = []
    for k in octs:
        rec = {"octaves": list(k), "fetch_bytes": fo.get(k), "write_bytes": wo.get(k)}
        rec["hbm_bytes"] = (fo.get(k) or 0.0) + (wo.get(k) or 0.0)
        if geo:
            rec["planes"] = [list(geo[4][o]) for o in k if o < len(geo[4])]
        po.append(rec)
    pass_bytes = (ftot or 0.0) + (wtot or 0.0) if (ftot is not None or wtot is not None) else None
    oct0 = next((r["hbm_bytes"] for r in po if r["octaves"] == [0]), None)
    out = {
        "config_key": a.config_key,
        "round": a.round,
        "generated_unix": int(time.time()),
        "pass_hbm_bytes": pass_bytes,
        "hbm_bytes_per_launch": oct0,
        "per_octave": po,
        "detections": {"fetch_run": nf, "write_run": nw},
        "kernel": "Gaussian+DoG pass: every pass launch of one detection (PASS_PREFIXES: k_gauss_*, k_seed_*, "
                  "k_upsample_base), octaves by launch order, helpers charged to the next tile launch; "
                  "hbm_bytes_per_launch = octave 0's launch",
        "launches": launches,
        "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate runs; per detection the pass's "
                  "consecutive launches on its queue, averaged over detections; bytes = 2 x FETCH_SIZE x 1024 + "
                  "WRITE_SIZE x 1024 (MI355X_MICROARCH.md, HBM); TA busy = TA_TA_BUSY_sum / (256 x "
                  "GRBM_GUI_ACTIVE / 8)",
    }
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    for r in launches:
        print("%-44s grid %9d  %8.1f MB read %8.1f MB written%s%s%s" % (
            r["kernel"][:44], r["grid"], (r["fetch_bytes"] or 0) / 1e6, (r["write_bytes"] or 0) / 1e6,
            "  TA busy %.2f" % r["ta_busy_frac"] if "ta_busy_frac" in r else "",
            "  L2 hit %.2f" % r["l2_hit_rate"] if "l2_hit_rate" in r else "",
            "  fp64 FMA issue %.2f" % r["fma_issue_frac"] if "fma_issue_frac" in r else ""))
    for r in po:
        print("octave %-6s %s  %8.1f MB read %8.1f MB written" % (
            ",".join(str(o) for o in r["octaves"]), r.get("planes"), (r["fetch_bytes"] or 0) / 1e6,
            (r["write_bytes"] or 0) / 1e6))
    print("pass: %.1f MB over %d / %d detections" % ((pass_bytes or 0) / 1e6, nf, nw))


if __name__ == "__main__":
    main()
