#!/usr/bin/env python3
"""Encode the configs[1] batch through lsm_encode_blocks (u64 offsets) and
lsm_encode_blocks32 (u32 offsets), alternating, for a rocprofv3 kernel trace
of both (the per-kernel durations of the two offset widths)."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
for p in (ROOT, ROOT / "lsm-tree_amd", ROOT / "oracle", ROOT / "tests"):
    sys.path.insert(0, str(p))
import torch  # noqa: E402
import bench  # noqa: E402
import lsmgpu  # noqa: E402

torch.cuda.set_device(0)
nb = 1 << 20
items, starts, n = bench.make_workload(torch, lsmgpu, nb)
items32 = dict(items, key_off=items["key_off"].to(torch.int32), val_off=items["val_off"].to(torch.int32))
enc = lsmgpu.Encoder()
out = enc.encode(items, starts, nb)
for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 5):
    enc.encode(items, starts, nb, out=out)
    enc.encode(items32, starts, nb, out=out)
torch.cuda.synchronize()
print("done")
