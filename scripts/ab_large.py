#!/usr/bin/env python3
"""Timing of the large-block legs (bench.bench_large_blocks shapes: 240 x 1 MiB,
60 x 4 MiB data blocks): encode, and decode with / without the huge-block
workspace pool.  Outputs of both decode paths are compared with each other
(parity against the oracle is tests/test_gpu_large_blocks.py's job).

usage: scripts/ab_large.py [--steps 5] [--which 1MiB,4MiB]
"""
import argparse
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
for p in (ROOT, ROOT / "lsm-tree_amd", ROOT / "oracle", ROOT / "tests"):
    sys.path.insert(0, str(p))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--which", default="1MiB,4MiB")
    a = ap.parse_args()
    import torch
    import bench
    import lsmgpu
    torch.cuda.set_device(0)
    shapes = {"1MiB": (240, 13108), "4MiB": (60, 52429), "256KiB": (960, 3277)}
    for name in a.which.split(","):
        nb, ipb = shapes[name]
        items, starts, n = bench.make_workload(torch, lsmgpu, nb, items_per_block=ipb, seed=0x5EED0007)
        enc_ctx = lsmgpu.Encoder()
        enc = enc_ctx.encode(items, starts, nb)
        torch.cuda.synchronize()
        total = int(enc["block_off"][nb].item())
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.steps):
            enc_ctx.encode(items, starts, nb, out=enc)
        e1.record()
        torch.cuda.synchronize()
        enc_ms = e0.elapsed_time(e1) / a.steps
        res = {}
        for pool in (True, False):
            dec = lsmgpu.Decoder()
            out = dec.alloc_outputs(n, nb)
            dec.decode(enc["buf"], enc["block_off"], nb, out, n, pool=pool)
            torch.cuda.synchronize()
            e0.record()
            for _ in range(a.steps):
                dec.decode(enc["buf"], enc["block_off"], nb, out, n, pool=pool)
            e1.record()
            torch.cuda.synchronize()
            assert int((out["status"][:nb] != 0).sum().item()) == 0
            res[pool] = (e0.elapsed_time(e1) / a.steps, out)
        same = all(bool((res[True][1][f][:n] == res[False][1][f][:n]).all().item()) for f in ("seqno", "key_off",
                                                                                             "val_off", "val_len"))
        gib = total / 2 ** 30
        print(f"{name}: {nb} blocks {total} B  encode {enc_ms:.3f} ms ({gib / enc_ms * 1e3:.1f} GiB/s)  "
              f"decode pool {res[True][0]:.3f} ms ({gib / res[True][0] * 1e3:.1f} GiB/s)  "
              f"no-pool {res[False][0]:.3f} ms ({gib / res[False][0] * 1e3:.1f} GiB/s)  same={same}", flush=True)
        del items, enc, res
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
