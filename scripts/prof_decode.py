#!/usr/bin/env python3
"""Run decode variants back to back for rocprofv3 PMC collection (diagnostic).

Dispatch order per round: full, no-parse, stage-only, no-hash (kernel
decode_blocks_kernel, item_start precomputed).  Use with e.g.
  rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU ... --output-format csv -d DIR -o pmc -- python scripts/prof_decode.py
"""
import argparse
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
for p in (ROOT, ROOT / "lsm-tree_amd", ROOT / "oracle", ROOT / "tests"):
    sys.path.insert(0, str(p))

import torch  # noqa: E402

import bench  # noqa: E402
import lsmgpu  # noqa: E402

VARIANTS = [("full", 0), ("no-parse", 0x200), ("stage-only", 0x700), ("no-hash", 0x100), ("phaseA-only", 0x800),
            ("stage-no-header", 0x1700), ("no-header-no-dma", 0x3700)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", type=int, default=1 << 18)
    ap.add_argument("--tuning", default="0,0,0", help="blocks_per_wave,stage_bytes,tile_items (0 = default)")
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--variants", default=",".join(v for v, _ in VARIANTS))
    args = ap.parse_args()
    torch.cuda.set_device(0)
    nb = args.blocks
    items, starts, n_items = bench.make_workload(torch, lsmgpu, nb)
    enc = lsmgpu.Encoder().encode(items, starts, nb)
    dec = lsmgpu.Decoder()
    out = dec.alloc_outputs(n_items, nb, fields=bench.DATA_FIELDS)  # the bench's data-block outputs (no handle_off)
    dec.decode(enc["buf"], enc["block_off"], nb, out, n_items)
    torch.cuda.synchronize()
    v = [int(x, 0) for x in args.tuning.split(",")]
    v = v + [0] * (4 - len(v))
    base, xf = tuple(v[:3]), v[3]
    chosen = [(v, f) for v, f in VARIANTS if v in args.variants.split(",")]
    for _ in range(args.reps):
        for name, fl in chosen:
            dec.decode(enc["buf"], enc["block_off"], nb, out, n_items, tuning=base + (1 | xf | fl,))
    torch.cuda.synchronize()
    print("variants:", [v for v, _ in chosen], "reps", args.reps, "blocks", nb, "bytes",
          int(enc["block_off"][nb].item()), "items", n_items)


if __name__ == "__main__":
    main()
