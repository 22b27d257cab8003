#!/usr/bin/env python3
"""Per-phase s_memtime totals of encode_huge_records_kernel, wave 0 of each
workgroup (diagnostic build: LSMGPU_LIB=lsm-tree_amd/.variants/libdiag.so,
lsm_block_params.reserved bit 0x40), on the bench's 1 MiB / 4 MiB batches."""
import ctypes as C
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
for p in (ROOT, ROOT / "lsm-tree_amd", ROOT / "oracle", ROOT / "tests"):
    sys.path.insert(0, str(p))

import torch  # noqa: E402

import bench  # noqa: E402
import lsmgpu  # noqa: E402

NAMES = {6: "loop / edges", 0: "unit lookup", 1: "records -> LDS", 2: "barrier", 3: "contributions",
         4: "copy-out", 5: "tail unit"}
torch.cuda.set_device(0)
L = lsmgpu.lib()
buf = (C.c_uint64 * 16)()
orig = lsmgpu.LsmBlockParams
for name, nb, ipb in (("1MiB", 240, 13108), ("4MiB", 60, 52429)):
    items, starts, n = bench.make_workload(torch, lsmgpu, nb, items_per_block=ipb, seed=0x5EED0007)
    enc = lsmgpu.Encoder()
    out = enc.encode(items, starts, nb)
    torch.cuda.synchronize()
    L.lsm_diag_encode_phases(buf)
    lsmgpu.LsmBlockParams = lambda ri, bt, c, r, hr: orig(ri, bt, c, 0x40, hr)
    enc.encode(items, starts, nb, out=out)
    torch.cuda.synchronize()
    lsmgpu.LsmBlockParams = orig
    L.lsm_diag_encode_phases(buf)
    cnt = max(1, buf[15])
    tot = sum(buf[i] for i in NAMES)
    print(f"{name}: {cnt} record units; ticks per unit, wave 0:")
    for i, nm in NAMES.items():
        print(f"  {nm:20s} {buf[i] / cnt:9.1f}  {100 * buf[i] / max(1, tot):5.1f}%")
    del items, out
    torch.cuda.empty_cache()
