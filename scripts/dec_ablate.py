#!/usr/bin/env python3
"""Decode group-kernel ablations (diagnostic build: LSMGPU_LIB=lsm-tree_amd/.variants/libdiag.so):
time lsm_decode_blocks on configs[1] with parts of the work skipped
(lsm_decode_tuning.flags diag bits, outputs invalid), to separate the memory
skeleton (stage DMA + barriers + stores) from the parse / hash compute."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
for p in (ROOT, ROOT / "lsm-tree_amd", ROOT / "oracle", ROOT / "tests"):
    sys.path.insert(0, str(p))

import torch  # noqa: E402

import bench  # noqa: E402
import lsmgpu  # noqa: E402

SKIP_HASH, SKIP_PARSE, SKIP_STORE, SKIP_PHASEB = 0x100, 0x200, 0x400, 0x800
VARIANTS = [("full", 0), ("no hash", SKIP_HASH), ("no stores", SKIP_STORE), ("no phase B", SKIP_PHASEB),
            ("no parse (A+B)", SKIP_PARSE), ("no hash, no stores", SKIP_HASH | SKIP_STORE),
            ("stage only (no hash, no parse)", SKIP_HASH | SKIP_PARSE)]
torch.cuda.set_device(0)
which = sys.argv[1] if len(sys.argv) > 1 else "c1"
shape = {"c1": dict(n_blocks=1 << 20), "c3": dict(n_blocks=262144, items_per_block=56, key_len=40, val_len=256,
                                                  kind="prefix")}[which]
items, starts, n = bench.make_workload(torch, lsmgpu, **shape)
nb = shape["n_blocks"]
enc = lsmgpu.Encoder().encode(items, starts, nb)
torch.cuda.synchronize()
del items
dec = lsmgpu.Decoder()
out = dec.alloc_outputs(n, nb, fields=bench.DATA_FIELDS)
dec.decode(enc["buf"], enc["block_off"], nb, out, n)
torch.cuda.synchronize()
res = {name: [] for name, _ in VARIANTS}
for _ in range(3):
    for name, fl in VARIANTS:
        tune = (0, 0, 0, lsmgpu.DECODE_ITEM_START_VALID | fl)
        dec.decode(enc["buf"], enc["block_off"], nb, out, n, tuning=tune)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            dec.decode(enc["buf"], enc["block_off"], nb, out, n, tuning=tune)
        e1.record()
        torch.cuda.synchronize()
        res[name].append(e0.elapsed_time(e1) / 10)
total = int(enc["block_off"][nb].item())
print(f"{which}: {nb} blocks, {total} bytes, {n} items (diagnostic build; min of 3 x 10 launches)")
for name, _ in VARIANTS:
    ms = min(res[name])
    print(f"  {name:32s} {ms:.4f} ms   read {total / ms / 1e6:.0f} GB/s")
