#!/usr/bin/env python3
"""Per-phase s_memtime totals of decode_big_kernel (diagnostic build:
LSMGPU_LIB=lsm-tree_amd/.variants/libdiag.so) on the configs[4] 64 KiB
segments."""
import ctypes as C
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
for p in (ROOT, ROOT / "lsm-tree_amd", ROOT / "oracle", ROOT / "tests"):
    sys.path.insert(0, str(p))

import torch  # noqa: E402

import bench  # noqa: E402
import lsmgpu  # noqa: E402

NAMES = {0: "wait DMA", 1: "header/trailer", 2: "owner fill", 3: "phase A | contribs", 4: "chain | phase B",
         5: "status", 6: "issue next DMA", 7: "next-block handle"}
torch.cuda.set_device(0)
L = lsmgpu.lib()
buf = (C.c_uint64 * 32)()
for bs, ipb, kind, est in bench.C5_SEGMENTS[4:]:
    nb = int((8 << 30) / 6 / est)
    items, starts, n = bench.make_workload(torch, lsmgpu, nb, items_per_block=ipb, kind=kind)
    enc = lsmgpu.Encoder().encode(items, starts, nb)
    dec = lsmgpu.Decoder()
    out = dec.alloc_outputs(n, nb, fields=bench.DATA_FIELDS)
    dec.decode(enc["buf"], enc["block_off"], nb, out, n)
    torch.cuda.synchronize()
    L.lsm_diag_decode_phases(buf)
    import os
    fl = int(os.environ.get("BIG_FLAGS", "0"), 0)
    dec.decode(enc["buf"], enc["block_off"], nb, out, n, tuning=(0, 0, 0, fl) if fl else None)
    torch.cuda.synchronize()
    L.lsm_diag_decode_phases(buf)
    cnt = max(1, buf[15])
    tot = sum(buf[i] for i in NAMES)
    print(f"{bs} {kind}: {cnt} blocks through the big kernel; ticks per block (wave 0):")
    for i, nm in NAMES.items():
        print(f"  {nm:20s} {buf[i] / cnt:9.0f}  {100 * buf[i] / max(1, tot):5.1f}%")
    del items, enc, out
    torch.cuda.empty_cache()
