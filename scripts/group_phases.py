#!/usr/bin/env python3
"""Per-phase s_memtime totals of decode_blocks_kernel (the group kernel;
diagnostic build: LSMGPU_LIB=lsm-tree_amd/.variants/libdiag.so) on the
configs[1] shape, configs[3] (16 KiB prefix) and the configs[4] 4/16 KiB
segments. Ticks are per group, wave 0 for the barrier phases; the role rows
are the mean over the waves that ran that role."""
import ctypes as C
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
for p in (ROOT, ROOT / "lsm-tree_amd", ROOT / "oracle", ROOT / "tests"):
    sys.path.insert(0, str(p))

import torch  # noqa: E402

import bench  # noqa: E402
import lsmgpu  # noqa: E402

torch.cuda.set_device(0)
L = lsmgpu.lib()
buf = (C.c_uint64 * 32)()
CASES = [("configs[1] 4K counter", 1 << 20, dict(items_per_block=52)),
         ("configs[3] 16K prefix", 262144, dict(items_per_block=56, key_len=40, val_len=256, kind="prefix")),
         ("4K random", 240000, dict(items_per_block=52, kind="random")),
         ("16K counter", 65536, dict(items_per_block=205, kind="counter")),
         ("16K random", 65536, dict(items_per_block=205, kind="random"))]
for name, nb, kw in CASES:
    items, starts, n = bench.make_workload(torch, lsmgpu, nb, **kw)
    enc = lsmgpu.Encoder().encode(items, starts, nb)
    dec = lsmgpu.Decoder()
    out = dec.alloc_outputs(n, nb, fields=bench.DATA_FIELDS)
    dec.decode(enc["buf"], enc["block_off"], nb, out, n)
    torch.cuda.synchronize()
    L.lsm_diag_decode_phases(buf)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    dec.decode(enc["buf"], enc["block_off"], nb, out, n)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1)
    L.lsm_diag_decode_phases(buf)
    g = buf[16:]
    groups = max(1, g[5])
    print(f"{name}: {nb} blocks, {ms:.3f} ms, {groups} groups ({g[6] / groups:.2f} blocks/group); "
          f"big kernel blocks {buf[15]}")
    for i, nm in enumerate(["wait DMA", "header/trailer", "phase A | hash", "phase B", "status + next DMA"]):
        print(f"  {nm:20s} {g[i] / groups:9.0f}")
    for i, nm in ((8, "role phase A"), (10, "role hash (wave/block)"), (12, "role hash (rows)")):
        c = max(1, g[i + 1])
        print(f"  {nm:24s} {g[i] / c:9.0f}  x{g[i + 1] / groups:.2f} per group")
    del items, enc, out
    torch.cuda.empty_cache()
