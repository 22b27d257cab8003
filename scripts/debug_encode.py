"""Debug helper: encode a random batch on GPU and oracle, report the first
differing block (offset, size, items) — test infrastructure (uses the oracle)."""
import random
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
for p in (ROOT / "lsm-tree_amd", ROOT / "oracle", ROOT / "tests"):
    sys.path.insert(0, str(p))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import lsmgpu  # noqa: E402
import pyoracle  # noqa: E402
from helpers import random_sorted_items  # noqa: E402

ri, ratio = int(sys.argv[1]), float(sys.argv[2])
items = random_sorted_items(3000, seed=ri * 7 + int(ratio), vmax=120)
rng = random.Random(ri)
starts = [0]
while starts[-1] < items.n:
    starts.append(min(items.n, starts[-1] + rng.randint(1, 120)))
starts = np.array(starts, np.uint32)
ref_buf, ref_off = pyoracle.encode_blocks(items, starts, restart_interval=ri, hash_ratio=ratio)
d = lsmgpu.items_to_device(items)
enc = lsmgpu.Encoder().encode(d, torch.from_numpy(starts.astype(np.int32)).cuda(), len(starts) - 1,
                              restart_interval=ri, hash_ratio=ratio)
torch.cuda.synchronize()
off = enc["block_off"].cpu().numpy().view(np.uint64)
buf = enc["buf"].cpu().numpy()
for b in range(len(starts) - 1):
    g = buf[off[b]:off[b + 1]].tobytes()
    r = ref_buf[ref_off[b]:ref_off[b + 1]].tobytes()
    if g != r:
        i = next(k for k in range(min(len(g), len(r))) if g[k] != r[k])
        tr = r[-31:]
        print(f"block {b}: items {starts[b]}..{starts[b+1]} size {len(r)} first diff at {i} (payload {i-33}); "
              f"trailer ri={tr[0]} step={tr[1]} bin_len={int.from_bytes(tr[2:6],'little')} "
              f"bin_off={int.from_bytes(tr[6:10],'little')} hash_len={int.from_bytes(tr[10:14],'little')} "
              f"hash_off={int.from_bytes(tr[14:18],'little')}")
        print("gpu", g[max(0, i - 8):i + 24].hex())
        print("ref", r[max(0, i - 8):i + 24].hex())
        pd = [k for k in range(33, min(len(g), len(r))) if g[k] != r[k]]
        print("payload diffs:", len(pd), "first", pd[:10], [(g[k], r[k]) for k in pd[:10]])
        nb = len(starts) - 1
        print("n_blocks", nb, "sizes around", [int(ref_off[x + 1] - ref_off[x]) for x in range(max(0, b - 3), min(nb, b + 3))])
        print("gpu stale:", g[33 + pd[0]:33 + pd[0] + 64].hex())
        for bb in range(b, min(nb, b + 4)):
            g2 = buf[off[bb]:off[bb + 1]].tobytes(); r2 = ref_buf[ref_off[bb]:ref_off[bb + 1]].tobytes()
            dd = [k for k in range(min(len(g2), len(r2))) if g2[k] != r2[k]]
            print("block", bb, "size", len(r2), "diffs", len(dd), "ranges", (dd[0], dd[-1]) if dd else None)
        break
else:
    print("all equal")
