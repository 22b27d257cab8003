#!/usr/bin/env python3
"""Encode ablations on a diagnostic build (LSMGPU_LIB=...libdiag.so): kernel
time with parts of the group kernel's record writer dropped (outputs invalid).
Bits (lsm_block_params.reserved, u8): 1 all record stores, 0x20 value copies,
0x40 key copies, 0x60 header varints, 2 hash/header, 4 copy-out."""
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parent.parent
for p in (ROOT, ROOT / "lsm-tree_amd", ROOT / "oracle", ROOT / "tests"):
    sys.path.insert(0, str(p))
import torch  # noqa: E402
import bench  # noqa: E402
import lsmgpu  # noqa: E402


def main():
    torch.cuda.set_device(0)
    which = sys.argv[1] if len(sys.argv) > 1 else "c1"
    if which == "c1":
        nb = 1 << 20
        items, starts, n = bench.make_workload(torch, lsmgpu, nb)
    else:
        nb = 262144
        items, starts, n = bench.make_workload(torch, lsmgpu, nb, items_per_block=56, key_len=40, val_len=256,
                                               kind="prefix")
    lsmgpu.lib()
    orig = lsmgpu.LsmBlockParams
    enc_ctx = lsmgpu.Encoder()
    enc = enc_ctx.encode(items, starts, nb)
    torch.cuda.synchronize()
    bits_list = [(0, "full"), (0x20, "no value copy"), (0x40, "no key copy"), (0x60, "no header varints"),
                 (1, "no record stores"), (2, "no hash/header"), (4, "no copy-out"),
                 (7, "none of records/hash/copy-out")]
    res = {b: [] for b, _ in bits_list}
    for r in range(3):
        for bits, name in bits_list:
            lsmgpu.LsmBlockParams = lambda ri, bt, c, rr, hr, bits=bits: orig(ri, bt, c, bits, hr)
            enc_ctx.encode(items, starts, nb, out=enc)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                enc_ctx.encode(items, starts, nb, out=enc)
            e1.record()
            torch.cuda.synchronize()
            res[bits].append(e0.elapsed_time(e1) / 5)
    lsmgpu.LsmBlockParams = orig
    for bits, name in bits_list:
        v = sorted(res[bits])[1]
        print(f"{which} {name:32s} {v:.4f} ms  (delta vs full {v - sorted(res[0])[1]:+.4f})")


if __name__ == "__main__":
    main()
