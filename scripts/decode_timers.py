#!/usr/bin/env python3
"""In-kernel phase timers of the decode kernel (diagnostic, tuning flag 0x2000).

Prints the average clock64() cycles per staged group for each phase, from the
point of view of the waves that ran it: form/dma/hdr/split/B/tail are summed
over all waves of a workgroup (÷ waves), A over the phase-A wave, hash over
the hash waves.
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

NAMES = ["form", "dma", "hdr", "A", "hash", "split", "B", "tail", "groups"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", type=int, default=1 << 18)
    ap.add_argument("--tuning", default="48,65536,1024")
    ap.add_argument("--waves", type=int, default=4)
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
    buf = (C.c_uint64 * 16)()
    base = [int(x, 0) for x in args.tuning.split(",")]
    for extra, label in ((0, "full"), (0x100, "no-hash"), (0x800, "no-phaseB"), (0x200, "no-parse")):
        lib.lsm_diag_decode_timers(buf, 16, 1)
        dec.decode(enc["buf"], enc["block_off"], nb, out, n_items, tuning=tuple(base[:3]) + (1 | 0x2000 | extra,))
        torch.cuda.synchronize()
        lib.lsm_diag_decode_timers(buf, 16, 1)
        t = list(buf)[:len(NAMES)]
        groups = t[8] / args.waves
        per = {n: t[i] / groups for i, n in enumerate(NAMES[:8])}
        for n in ("form", "dma", "hdr", "split", "B", "tail"):
            per[n] /= args.waves
        per["hash"] /= (args.waves - 1)
        print(f"{label:10s} groups {groups:9.0f}  " + "  ".join(f"{n} {per[n]:8.0f}" for n in NAMES[:8]), flush=True)


if __name__ == "__main__":
    main()
