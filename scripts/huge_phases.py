#!/usr/bin/env python3
"""Per-phase s_memtime totals of decode_huge_kernel, wave 0 of each workgroup
(diagnostic build: LSMGPU_LIB=lsm-tree_amd/.variants/libdiag.so), on the
bench's 1 MiB / 4 MiB large-block batches."""
import ctypes as C
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
for p in (ROOT, ROOT / "lsm-tree_amd", ROOT / "oracle", ROOT / "tests"):
    sys.path.insert(0, str(p))

import torch  # noqa: E402

import bench  # noqa: E402
import lsmgpu  # noqa: E402

NAMES = {6: "unit lookup", 0: "DMA issue + r0/r1", 1: "fast check, bix, meta", 2: "wait DMA", 3: "phase A",
         4: "contributions", 5: "phase B / walk"}
torch.cuda.set_device(0)
L = lsmgpu.lib()
buf = (C.c_uint64 * 32)()
for name, nb, ipb in (("1MiB", 240, 13108), ("4MiB", 60, 52429)):
    items, starts, n = bench.make_workload(torch, lsmgpu, nb, items_per_block=ipb, seed=0x5EED0007)
    enc = lsmgpu.Encoder().encode(items, starts, nb)
    dec = lsmgpu.Decoder()
    out = dec.alloc_outputs(n, nb)
    dec.decode(enc["buf"], enc["block_off"], nb, out, n, pool=True)
    torch.cuda.synchronize()
    L.lsm_diag_decode_phases(buf)
    dec.decode(enc["buf"], enc["block_off"], nb, out, n, pool=True)
    torch.cuda.synchronize()
    L.lsm_diag_decode_phases(buf)
    cnt = max(1, buf[15])
    tot = sum(buf[8 + i] for i in NAMES)
    print(f"{name}: {cnt} units; ticks (s_memtime, 100 MHz) per unit, wave 0:")
    for i, nm in NAMES.items():
        print(f"  {nm:24s} {buf[8 + i] / cnt:9.1f}  {100 * buf[8 + i] / max(1, tot):5.1f}%")
    del items, enc, out
    torch.cuda.empty_cache()
