#!/usr/bin/env python3
"""LDS-DMA streaming ceiling (diagnostic): GB/s of lsm_diag_dma_probe over a
4 GiB device buffer for loader-wave counts, in-flight limits and address forms."""
import ctypes as C
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "lsm-tree_amd"))

import torch  # noqa: E402

import lsmgpu  # noqa: E402


def main():
    torch.cuda.set_device(0)
    nbytes = 4 << 30
    buf = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    buf.fill_(1)
    lib = lsmgpu.lib()
    lib.lsm_diag_dma_probe.argtypes = [C.c_void_p, C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32, C.c_void_p]
    cases = [(1, 1, 48), (1, 0, 48), (1, 3, 48), (1, 1, 24), (1, 1, 12), (2, 1, 24), (2, 1, 48), (4, 1, 16),
             (4, 1, 32), (8, 1, 8), (8, 1, 16), (16, 1, 8)]
    for loaders, mode, infl in cases:
        times = []
        for _ in range(4):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            rc = lib.lsm_diag_dma_probe(buf.data_ptr(), nbytes, loaders, mode, infl, None)
            e1.record()
            torch.cuda.synchronize()
            assert rc == 0
            times.append(e0.elapsed_time(e1))
        ms = min(times[1:])
        print(f"loaders {loaders:2d} mode {mode} ({'saddr' if mode & 1 else 'vaddr'}{' nt' if mode & 2 else ''}) "
              f"inflight {infl:2d}: {ms:7.3f} ms  {nbytes / ms / 1e6:7.1f} GB/s", flush=True)


if __name__ == "__main__":
    main()
