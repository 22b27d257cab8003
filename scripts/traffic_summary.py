#!/usr/bin/env python3
"""HBM traffic per decode launch from two rocprofv3 PMC passes (FETCH_SIZE,
WRITE_SIZE) over scripts/prof_decode.py --variants full.

gfx950 correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE reports half
the bytes of wide streaming reads -> doubled.  WRITE_SIZE is exact for 16-B
stores; our SoA stores are 1-8 B per lane (uncalibrated), reported raw.
Usage: traffic_summary.py FETCH_DIR WRITE_DIR BLOCKS BYTES ITEMS > profiles/traffic_rNN.json
"""
import csv
import json
import sys
from pathlib import Path


def per_dispatch(d, counter):
    vals = {}
    for f in Path(d).rglob("*counter_collection.csv"):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if ("decode_blocks_kernel" in r.get("Kernel_Name", "") or "decode_ring_kernel" in r.get("Kernel_Name", "")) and r["Counter_Name"] == counter:
                    k = int(r["Dispatch_Id"])
                    vals[k] = vals.get(k, 0.0) + float(r["Counter_Value"])
    keys = sorted(vals)[1:]  # first dispatch: warm-up decode (computes item_start)
    return [vals[k] for k in keys]


def main():
    fdir, wdir, blocks, nbytes, items = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])
    f = per_dispatch(fdir, "FETCH_SIZE")
    w = per_dispatch(wdir, "WRITE_SIZE")
    fk = sum(f) / len(f)
    wk = sum(w) / len(w)
    alg = nbytes + items * 25 + blocks * 8
    out = {
        "kernel": "decode_blocks_kernel", "blocks": blocks, "input_bytes": nbytes, "items": items,
        "dispatches": len(f), "fetch_size_kb_raw": round(fk, 1), "write_size_kb_raw": round(wk, 1),
        "read_bytes_per_launch": int(2 * fk * 1024), "write_bytes_per_launch": int(wk * 1024),
        "bytes_per_launch": int(2 * fk * 1024 + wk * 1024), "alg_bytes_per_launch": alg,
        "traffic_over_alg": round((2 * fk * 1024 + wk * 1024) / alg, 4),
        "note": "FETCH_SIZE x2 (gfx950 wide-read correction); WRITE_SIZE raw (1-8 B/lane stores, uncalibrated)",
    }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
