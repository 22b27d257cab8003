#!/usr/bin/env python3
"""Encode loop on the bench workload (for rocprofv3 --kernel-trace --stats)."""
import argparse
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
for p in (ROOT, ROOT / "lsm-tree_amd", ROOT / "oracle", ROOT / "tests"):
    sys.path.insert(0, str(p))

import torch  # noqa: E402

import bench  # noqa: E402
import lsmgpu  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", type=int, default=1 << 20)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--workload", default="counter", choices=["counter", "prefix16k"])
    ap.add_argument("--off64", action="store_true", help="u64 key / value offsets (lsm_encode_blocks); default: "
                    "u32 (lsm_encode_blocks32), as bench.py's timed step")
    ap.add_argument("--diag-bits", type=int, default=0, help="lsm_block_params.reserved for the timed loop (diagnostic build)")
    ap.add_argument("--phases", action="store_true", help="per-phase cycles of the group kernel (diagnostic build)")
    ap.add_argument("--ablate", action="store_true", help="diagnostic ablations (lsm_block_params.reserved bits)")
    args = ap.parse_args()
    torch.cuda.set_device(0)
    nb = args.blocks
    if args.workload == "counter":
        items, starts, n_items = bench.make_workload(torch, lsmgpu, nb)
    else:
        items, starts, n_items = bench.make_workload(torch, lsmgpu, nb, items_per_block=56, key_len=40, val_len=256)
    off_bytes = 8 if args.off64 else 4
    # (the arena sizes from the u64 offsets: a u32 offset past 2^31 reads back negative)
    key_val = int(items["key_off"][n_items].item()) + int(items["val_off"][n_items].item())
    if not args.off64:
        items = dict(items, key_off=items["key_off"].to(torch.int32), val_off=items["val_off"].to(torch.int32))
    if args.diag_bits:
        lsmgpu.lib()
        orig_p = lsmgpu.LsmBlockParams
        lsmgpu.LsmBlockParams = lambda ri, bt, c, r, hr, *f: orig_p(ri, bt, c, args.diag_bits, hr, *f)
    enc_ctx = lsmgpu.Encoder()
    enc = enc_ctx.encode(items, starts, nb)
    torch.cuda.synchronize()
    total = int(enc["block_off"][nb].item())
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(args.reps):
        enc_ctx.encode(items, starts, nb, out=enc)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / args.reps
    assert int((enc["status"][:nb] != 0).sum()) == 0
    if args.phases:
        import ctypes as C
        L = lsmgpu.lib()
        orig = lsmgpu.LsmBlockParams
        lsmgpu.LsmBlockParams = lambda ri, bt, c, r, hr, *f: orig(ri, bt, c, 0x80, hr, *f)
        buf = (C.c_uint64 * 16)()
        rc0 = L.lsm_diag_encode_phases(buf)
        enc_ctx.encode(items, starts, nb, out=enc)
        torch.cuda.synchronize()
        rc1 = L.lsm_diag_encode_phases(buf)
        print("phase readout rc", rc0, rc1, "status nonzero", int((enc["status"][:nb] != 0).sum()), list(buf))
        lsmgpu.LsmBlockParams = orig
        n = max(1, buf[15])
        names = {11: "kernel start", 0: "loop top", 9: "next items issue", 1: "setup", 2: "scan", 3: "records",
                 10: "next DMA issue", 4: "tails", 5: "hash", 6: "scramble+hdr", 7: "wait", 8: "copy-out"}
        tot = sum(buf[i] for i in names)
        print(f"group iterations {n}; s_memtime ticks per iteration (wave 0):")
        for i, nm in names.items():
            print(f"  {nm:16s} {buf[i] / n:9.0f}  {100 * buf[i] / max(1, tot):5.1f}%")
    if args.ablate:
        import ctypes as C
        L = lsmgpu.lib()
        for bits, name in ((1, "no record stores"), (2, "no hash/header"), (4, "no copy-out"), (7, "none of them"),
                           (8, "no group compute"), (12, "no compute/copy-out"), (16, "no next-group DMA"),
                           (28, "barriers + item loads")):
            orig = lsmgpu.LsmBlockParams
            class P2(C.Structure):  # noqa: E306
                _fields_ = orig._fields_
            def mk(ri, bt, c, r, hr, *f, bits=bits):
                return orig(ri, bt, c, bits, hr, *f)
            lsmgpu.LsmBlockParams = mk
            enc_ctx.encode(items, starts, nb, out=enc)
            torch.cuda.synchronize()
            e0.record()
            for _ in range(args.reps):
                enc_ctx.encode(items, starts, nb, out=enc)
            e1.record()
            torch.cuda.synchronize()
            lsmgpu.LsmBlockParams = orig
            print(f"  ablate {name:20s} {e0.elapsed_time(e1) / args.reps:.3f} ms", flush=True)
    alg = key_val + n_items * (bench.ENC_IN_PER_ITEM - 2 * (8 - off_bytes)) + 4 * (nb + 1) + total + 8 * (nb + 1) + 4 * nb
    print(f"encode {args.workload} (u{8 * off_bytes} offsets): {nb} blocks {n_items} items {total} bytes  {ms:.3f} ms  "
          f"{total / ms / 1e6:.1f} GB/s written  alg_bytes {alg}", flush=True)


if __name__ == "__main__":
    main()
