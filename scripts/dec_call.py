#!/usr/bin/env python3
"""The configs[1] decode timed as the kernel alone (item_start precomputed) and as
the whole lsm_decode_blocks call, in one process, after a fresh encode and after
another decode (HIP events, 10 calls each)."""
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
encoder = lsmgpu.Encoder()
enc = encoder.encode(items, starts, nb)
dec = lsmgpu.Decoder()
out = dec.alloc_outputs(n, nb, fields=bench.DATA_FIELDS)
valid = (0, 0, 0, lsmgpu.DECODE_ITEM_START_VALID)


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


for _ in range(2):
    k = timed(lambda: dec.decode(enc["buf"], enc["block_off"], nb, out, n, tuning=valid))
    c = timed(lambda: dec.decode(enc["buf"], enc["block_off"], nb, out, n))
    ec = timed(lambda: (encoder.encode(items, starts, nb, out=enc), dec.decode(enc["buf"], enc["block_off"], nb, out, n)))
    e = timed(lambda: encoder.encode(items, starts, nb, out=enc))
    print(f"kernel {k:.4f} ms  call {c:.4f} ms  encode+call {ec:.4f} ms  encode {e:.4f} ms  -> call after encode "
          f"{ec - e:.4f} ms", flush=True)
