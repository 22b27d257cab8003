#!/usr/bin/env python3
"""HBM traffic per launch from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE),
one entry per hot-path kernel group, in the format bench.load_traffic reads.

gfx950 correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE reports half
the bytes of wide streaming reads -> doubled.  Calibrated for every read shape
these kernels use (scripts/fetch_calib.py, profiles/r05_fetch_calib.json: u64,
u32 and u8 per lane, the plan's overlapping u64 windows, 16 B per lane and the
LDS-DMA all report exactly half).  WRITE_SIZE is exact for 16-B stores, u32
stores (r05_fetch_calib.json) and the decode SoA's 1-8 B stores
(scripts/write_calib.py, round 2).
Usage: traffic_summary.py DEC_FETCH DEC_WRITE DEC_BLOCKS DEC_BYTES DEC_ITEMS
                          ENC_FETCH ENC_WRITE ENC_ALG_BYTES ITEMS KEY_BYTES VAL_BYTES [OFF_BYTES]
                          > profiles/traffic_rNN.json
(OFF_BYTES: the width of the encode's key / value offsets, 8 or 4 (lsm_encode_blocks32); default 8)
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
                                         "FETCH_SIZE x2 (gfx950 correction, calibrated for LDS-DMA reads); WRITE_SIZE "
                                         "raw (1-8 B/lane SoA stores: exact, scripts/write_calib.py)")}
    if len(a) >= 8:
        names = ["encode_plan", "scan_tile", "encode_group_kernel", "encode_write_list", "encode_large"]
        f, n = per_dispatch(a[5], "FETCH_SIZE", names, True)
        w, _ = per_dispatch(a[6], "WRITE_SIZE", names, True)
        out["lsm_encode_blocks"] = entry("lsm_encode_blocks", f, w, n, dblocks, int(a[7]),
                                         "plan + scan + group kernels summed per launch; FETCH_SIZE x2 and WRITE_SIZE "
                                         "raw, both calibrated (profiles/r05_fetch_calib.json)")
        # per kernel: what each pass of the two-pass design must move (bytes per launch):
        #   plan  reads the item SoA (8 + 8 + 8 + 1 B; 4 + 4 + 8 + 1 with u32 offsets) and each key's first 16 bytes,
        #         writes erec (4 B per item) and per block size, plan, key / value span starts (40 B)
        #   group reads keys, values, the item SoA again, erec, the block plans (40 B) and offsets,
        #         writes the blocks and their statuses
        items, key_bytes, val_bytes = int(a[8]), int(a[9]), int(a[10])
        soa = 25 - 2 * (8 - (int(a[11]) if len(a) > 11 else 8))  # item SoA bytes per item
        out_bytes = int(a[7]) - (key_bytes + val_bytes + items * soa + 16 * dblocks + 4)
        plan_alg = items * (soa + 16 + 4) + dblocks * 40
        group_alg = key_bytes + val_bytes + items * (soa + 4) + dblocks * 48 + out_bytes
        for k, alg in (("encode_plan_wave_kernel", plan_alg), ("encode_group_kernel", group_alg)):
            f1, n1 = per_dispatch(a[5], "FETCH_SIZE", [k], True)
            w1, _ = per_dispatch(a[6], "WRITE_SIZE", [k], True)
            e = entry(k, f1, w1, n1, dblocks, alg, "this kernel's share of the two-pass encode; alg = the bytes its "
                                                   "pass must move (see traffic_summary.py)")
            out[k] = e
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
