#!/usr/bin/env python3
"""Role timers of the ring decode kernel (diagnostic, tuning flag 0x2000).

Prints, per workgroup (grid = one per CU), the microseconds each role spent
busy / idle over one launch (shader clock assumed 2.4 GHz), and the mean
issue -> publish latency of a group's LDS-DMA.
"""
import argparse
import ctypes as C
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
for p in (ROOT, ROOT / "lsm-tree_amd", ROOT / "oracle", ROOT / "tests"):
    sys.path.insert(0, str(p))

import torch  # noqa: E402

import bench  # noqa: E402
import lsmgpu  # noqa: E402

NAMES = ["L_issue", "L_wait", "L_idle", "land", "groups", "X_busy", "X_idle", "H_busy", "H_idle", "B_busy", "B_idle"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", type=int, default=1 << 20)
    ap.add_argument("--tunings", default="0,32768,512;0,32768,512,0,4,2,5")
    ap.add_argument("--clock-ghz", type=float, default=2.4)
    args = ap.parse_args()
    torch.cuda.set_device(0)
    nb = args.blocks
    items, starts, n_items = bench.make_workload(torch, lsmgpu, nb)
    enc = lsmgpu.Encoder().encode(items, starts, nb)
    dec = lsmgpu.Decoder()
    out = dec.alloc_outputs(n_items, nb)
    dec.decode(enc["buf"], enc["block_off"], nb, out, n_items)
    torch.cuda.synchronize()
    lib = lsmgpu.lib()
    lib.lsm_diag_decode_timers.argtypes = [C.POINTER(C.c_uint64), C.c_int, C.c_int]
    buf = (C.c_uint64 * 32)()
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    for t in args.tunings.split(";"):
        v = [int(x, 0) for x in t.split(",")] + [0] * 8
        v = v[:8]
        slots, nx, nh, nl = v[4] or 4, v[5] or 3, v[6] or 4, v[7] or 4
        nbw = 16 - nl - nx - nh
        for extra, label in ((0, "full"), (0x700, "stage-only")):
            tun = tuple(v[:3]) + (v[3] | 1 | 0x2000 | 0x80000 | extra,) + tuple(v[4:8])
            lib.lsm_diag_decode_timers(buf, 32, 1)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            dec.decode(enc["buf"], enc["block_off"], nb, out, n_items, tuning=tun)
            e1.record()
            torch.cuda.synchronize()
            lib.lsm_diag_decode_timers(buf, 32, 1)
            r = dict(zip(NAMES, list(buf)[16:16 + len(NAMES)]))
            us = lambda c, waves: c / args.clock_ghz / 1e3 / cus / waves  # noqa: E731
            groups = r["groups"] / cus / nl
            print(f"{t:28s} {label:10s} {e0.elapsed_time(e1):7.3f} ms  groups/WG {groups:6.0f}  "
                  f"L issue {us(r['L_issue'], nl):7.1f} wait {us(r['L_wait'], nl):7.1f} idle {us(r['L_idle'], nl):7.1f} | "
                  f"X busy {us(r['X_busy'], nx):7.1f} idle {us(r['X_idle'], nx):7.1f} | "
                  f"H busy {us(r['H_busy'], nh):7.1f} idle {us(r['H_idle'], nh):7.1f} | "
                  f"B busy {us(r['B_busy'], nbw):7.1f} idle {us(r['B_idle'], nbw):7.1f}  (us per wave)", flush=True)


if __name__ == "__main__":
    main()
