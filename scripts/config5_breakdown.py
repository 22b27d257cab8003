#!/usr/bin/env python3
"""configs[4] mixed batch: decode time per segment (diagnostic)."""
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
    import os
    cases = [(bs, (8 << 30) // 6 // est, dict(items_per_block=ipb, kind=kind)) for bs, ipb, kind, est in bench.C5_SEGMENTS]
    if os.environ.get("C5_EXTRA"):  # configs[1] and configs[3] shapes too
        cases = [(4096, 1 << 20, dict(items_per_block=52)),
                 (16384, 262144, dict(items_per_block=56, key_len=40, val_len=256, kind="prefix"))] + cases
    for bs, nb, kw in cases:
        kind = kw.get("kind", "counter") + ("" if kw.get("val_len", 64) == 64 else "-c3")
        nb = int(nb)
        items, starts, n = bench.make_workload(torch, lsmgpu, nb, **kw)
        enc = lsmgpu.Encoder().encode(items, starts, nb)
        torch.cuda.synchronize()
        total = int(enc["block_off"][nb].item())
        for tun in (None, (0, 0, 0, lsmgpu.DECODE_ITEM_START_VALID)):
            dec = lsmgpu.Decoder()
            out = dec.alloc_outputs(n, nb, fields=bench.DATA_FIELDS)
            dec.decode(enc["buf"], enc["block_off"], nb, out, n)
            torch.cuda.synchronize()
            assert int((out["status"][:nb] != 0).sum().item()) == 0
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                dec.decode(enc["buf"], enc["block_off"], nb, out, n, tuning=tun)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / 5
            print(f"{bs:6d} {kind:8s} blocks {nb:8d} bytes {total:11d} B/blk {total / nb:8.0f}  "
                  f"{'step' if tun is None else 'kernels'} {ms:7.3f} ms {total / ms / 1e6:8.1f} GB/s", flush=True)
        del items, enc, out
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
