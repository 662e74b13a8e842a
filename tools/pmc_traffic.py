#!/usr/bin/env python3
"""HBM bytes per launch of one kernel from two rocprofv3 --pmc passes
(FETCH_SIZE and WRITE_SIZE, KiB per dispatch), with the gfx950 correction of
MI355X_MICROARCH.md (FETCH_SIZE reports half the bytes of wide streaming
reads: doubled).  Writes the JSON bench.py reads as roofline.traffic.

usage: tools/pmc_traffic.py --kernel SUBSTR --config-key KEY --out FILE FETCH_DIR WRITE_DIR
"""
import argparse
import csv
import glob
import json
import os


def per_dispatch(d, counter, kernel):
    vals = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter and kernel in r["Kernel_Name"]:
                vals.append(float(r["Counter_Value"]))
    if not vals:
        raise SystemExit("no %s samples for kernel %r under %s" % (counter, kernel, d))
    return sum(vals) / len(vals), len(vals)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--config-key", required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    a = ap.parse_args()
    fk, nf = per_dispatch(a.fetch_dir, "FETCH_SIZE", a.kernel)
    wk, nw = per_dispatch(a.write_dir, "WRITE_SIZE", a.kernel)
    fetch = 2.0 * fk * 1024.0   # gfx950: FETCH_SIZE counts half of wide streaming reads
    write = wk * 1024.0
    out = {
        "config_key": a.config_key,
        "kernel": a.kernel,
        "fetch_size_kib": fk,
        "write_size_kib": wk,
        "dispatches": [nf, nw],
        "hbm_read_bytes_per_launch": fetch,
        "hbm_write_bytes_per_launch": write,
        "hbm_bytes_per_launch": fetch + write,
        "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes; "
                  "bytes = 2 x FETCH_SIZE x 1024 + WRITE_SIZE x 1024 (MI355X_MICROARCH.md, HBM)",
    }
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
