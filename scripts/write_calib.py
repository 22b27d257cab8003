#!/usr/bin/env python3
"""WRITE_SIZE calibration for the decode's SoA store shape (diagnostic).

Writes the parsed-item SoA of 54.5 M items (the configs[1] decode output)
with the decode kernel's per-lane 1-8 B stores and, for comparison, as
16 B/lane stores of the same bytes.  Run under rocprofv3 --pmc WRITE_SIZE
(and --kernel-trace for the times): bytes per launch = 25 * n exactly."""
import ctypes as C
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
lib = C.CDLL(str(ROOT / "lsm-tree_amd" / "ceiling" / "liblsmceiling.so"))
n = 54525952
buf = torch.empty(25 * n, dtype=torch.uint8, device="cuda")
s = torch.cuda.current_stream().cuda_stream
for mode in (0, 1):
    for _ in range(3):
        assert lib.lsm_ceiling_soa(C.c_void_p(buf.data_ptr()), C.c_uint64(n), mode, C.c_void_p(s)) == 0
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        lib.lsm_ceiling_soa(C.c_void_p(buf.data_ptr()), C.c_uint64(n), mode, C.c_void_p(s))
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 5
    print(f"mode {mode}: {25 * n} bytes  {ms:.4f} ms  {25 * n / ms / 1e6:.1f} GB/s", flush=True)
