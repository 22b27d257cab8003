"""LZ4 decompress timing on liblz4-compressed configs[1]-shaped blocks (diagnostic;
compare the default library with a variant, e.g. -DLSM_LZ4_DIAG_SKIP_DECODE).
usage: [LSMGPU_LIB=variant.so] python scripts/lz4_ablation.py [n_blocks]"""
import json
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "lsm-tree_amd"), str(ROOT)]
import lsmgpu  # noqa: E402
import bench  # noqa: E402

nb = int(sys.argv[1]) if len(sys.argv) > 1 else 131072
items, starts, n = bench.make_workload(torch, lsmgpu, nb)
enc = lsmgpu.Encoder().encode(items, starts, nb)
torch.cuda.synchronize()
r = bench.bench_lz4(torch, lsmgpu, enc, nb, reps=10, sample=nb)
print(json.dumps({"lib": str(lsmgpu.LIB_PATH), **r}))
