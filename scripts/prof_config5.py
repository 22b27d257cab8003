#!/usr/bin/env python3
"""configs[4] mixed batch (one rank's 8 GiB of 4/16/64 KiB data + index
blocks) decoded a few times, for rocprofv3 --kernel-trace --stats (diagnostic)."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
for p in (ROOT, ROOT / "lsm-tree_amd", ROOT / "oracle", ROOT / "tests"):
    sys.path.insert(0, str(p))

import torch  # noqa: E402

import bench  # noqa: E402
import lsmgpu  # noqa: E402

torch.cuda.set_device(0)
blocks, boff, nb, n_items, nbytes, n_idx, _ = bench.build_config5_shard(torch, lsmgpu, 8 << 30, 0, 16)
ms, out = bench.time_decode(torch, lsmgpu, blocks, boff, nb, n_items, 5, fields=bench.DATA_FIELDS + ["handle_off"])
print(f"config5: {nb} blocks ({n_idx} index) {nbytes} bytes  {ms:.3f} ms  {nbytes / ms / 1e6:.1f} GB/s", flush=True)
