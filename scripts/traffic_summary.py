#!/usr/bin/env python3
"""HBM traffic per launch from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE),
one entry per hot-path kernel group, in the format bench.load_traffic reads.

gfx950 correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE reports half
the bytes of wide streaming reads -> doubled.  WRITE_SIZE is exact for 16-B
stores; narrower stores (the decode SoA's 1-8 B lanes, the encode plan's u32
words) are uncalibrated and reported raw.
Usage: traffic_summary.py DEC_FETCH DEC_WRITE DEC_BLOCKS DEC_BYTES DEC_ITEMS
                          ENC_FETCH ENC_WRITE ENC_ALG_BYTES > profiles/traffic_rNN.json
"""
import csv
import json
import sys
from pathlib import Path


def per_dispatch(d, counter, names, skip_first):
    """Sum of `counter` per launch over kernels whose name contains any of `names`;
    consecutive dispatches of the group (plan + write kernels) form one launch."""
    rows = []
    for f in Path(d).rglob("*counter_collection.csv"):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if r["Counter_Name"] == counter and any(n in r.get("Kernel_Name", "") for n in names):
                    rows.append((int(r["Dispatch_Id"]), r["Kernel_Name"], float(r["Counter_Value"])))
    by = {}
    for did, name, v in rows:
        by.setdefault((did, name), 0.0)
        by[(did, name)] += v
    first = names[0]
    launches, cur = [], None
    for (did, name), v in sorted(by.items()):
        if first in name:
            cur = [v]
            launches.append(cur)
        elif cur is not None:
            cur.append(v)
    vals = [sum(x) for x in launches][1 if skip_first else 0:]
    return sum(vals) / len(vals), len(vals)


def entry(kernel, fetch_kb, write_kb, dispatches, blocks, alg, note):
    rd, wr = int(2 * fetch_kb * 1024), int(write_kb * 1024)
    return {"kernel": kernel, "blocks": blocks, "dispatches": dispatches, "fetch_size_kb_raw": round(fetch_kb, 1),
            "write_size_kb_raw": round(write_kb, 1), "read_bytes_per_launch": rd, "write_bytes_per_launch": wr,
            "bytes_per_launch": rd + wr, "alg_bytes_per_launch": alg, "traffic_over_alg": round((rd + wr) / alg, 4),
            "note": note}


def main():
    a = sys.argv[1:]
    dblocks, dbytes, ditems = int(a[2]), int(a[3]), int(a[4])
    f, n = per_dispatch(a[0], "FETCH_SIZE", ["decode_blocks_kernel"], True)
    w, _ = per_dispatch(a[1], "WRITE_SIZE", ["decode_blocks_kernel"], True)
    out = {"decode_blocks_kernel": entry("decode_blocks_kernel", f, w, n, dblocks, dbytes + ditems * 25 + dblocks * 8,
                                         "FETCH_SIZE x2 (gfx950 wide-read correction); WRITE_SIZE raw (1-8 B/lane "
                                         "SoA stores, uncalibrated)")}
    if len(a) >= 8:
        names = ["encode_plan", "scan_tile", "encode_group_kernel", "encode_write_list", "encode_large"]
        f, n = per_dispatch(a[5], "FETCH_SIZE", names, True)
        w, _ = per_dispatch(a[6], "WRITE_SIZE", names, True)
        out["lsm_encode_blocks"] = entry("lsm_encode_blocks", f, w, n, dblocks, int(a[7]),
                                         "plan + scan + group kernels summed per launch; FETCH_SIZE x2; WRITE_SIZE "
                                         "raw (16 B/lane copy-out exact, plan words uncalibrated)")
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
