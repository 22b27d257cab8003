#!/usr/bin/env python3
"""Experiment: lsm_encode_blocks / lsm_decode_blocks captured into a HIP graph
(torch.cuda.CUDAGraph) and replayed; prints the statuses and whether the
bytes match an eager call.  Batches: 4 KiB blocks (no pool) and an E1p batch
with huge blocks (pool)."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
for p in (ROOT, ROOT / "lsm-tree_amd", ROOT / "oracle", ROOT / "tests"):
    sys.path.insert(0, str(p))

import numpy as np
import torch

import lsmgpu
from helpers import counter_items


def run(name, sizes, pool, seed=5, tomb=0.0, replays=1):
    items = counter_items(int(sum(sizes)), seed=seed, tomb_frac=tomb)
    starts = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int32)
    d_items = lsmgpu.items_to_device(items)
    d_starts = torch.from_numpy(starts).cuda()
    nb = len(sizes)
    enc = lsmgpu.Encoder()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        out = enc.encode(d_items, d_starts, nb, pool=pool)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    ref = out["buf"].clone()
    ref_off = out["block_off"].clone()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        enc.encode(d_items, d_starts, nb, out=out, pool=pool)
    for r in range(replays):
        out["buf"].zero_()
        out["status"].fill_(-1)
        g.replay()
        torch.cuda.synchronize()
        st = out["status"][:nb].cpu().numpy()
        same = bool(torch.equal(out["buf"], ref)) and bool(torch.equal(out["block_off"], ref_off))
        print(f"{name} replay {r}: statuses {np.unique(st, return_counts=True)} same={same}", flush=True)


def main():
    torch.cuda.set_device(0)
    run("4KiB x 64 (no pool)", [52] * 64, False)
    run("E1p mixed (no pool)", [50, 200, 20000, 7, 1, 30000, 300, 13, 9000], False)
    run("E1p mixed (pool)", [50, 200, 20000, 7, 1, 30000, 300, 13, 9000], True)
    run("1 MiB x 4 (pool)", [13108] * 4, True)
    t = [50, 200, 20000, 7, 1, 30000, 300, 13, 9000, 64, 65, 129, 2500, 16400]
    run("test batch (pool)", t, True, seed=31, tomb=0.05, replays=2)
    run("test batch (no pool)", t, False, seed=31, tomb=0.05, replays=2)
    run("test batch no tombs (pool)", t, True, seed=31, replays=2)


if __name__ == "__main__":
    main()
