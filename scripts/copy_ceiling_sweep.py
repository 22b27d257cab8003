#!/usr/bin/env python3
"""Copy-ceiling variants (diagnostic): grid-stride 4-deep vs one 64 KiB tile
per workgroup (plain / non-temporal stores), 4 GiB, HIP events."""
import ctypes as C
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
lib = C.CDLL(str(ROOT / "lsm-tree_amd" / "ceiling" / "liblsmceiling.so"))
lib.lsm_ceiling_copy_variant.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_int, C.c_void_p]
n = 4 << 30
src = torch.empty(n, dtype=torch.uint8, device="cuda")
dst = torch.empty(n, dtype=torch.uint8, device="cuda")
s = torch.cuda.current_stream().cuda_stream
for v in (0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 1, 2):
    assert lib.lsm_ceiling_copy_variant(src.data_ptr(), dst.data_ptr(), n, v, s) == 0
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        lib.lsm_ceiling_copy_variant(src.data_ptr(), dst.data_ptr(), n, v, s)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 10
    print(f"variant {v}: {ms:.3f} ms  {2 * n / ms / 1e6:.1f} GB/s (read + write)", flush=True)
