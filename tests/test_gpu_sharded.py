"""Single-process multi-device encode / decode: a host write
buffer split at block cuts into shards balanced by key + value bytes
(lsmgpu.shard_items), each shard encoded on its device, the shards placed by
the exclusive scan of their byte totals; a host block buffer split into
byte-balanced shards (lsmgpu.shard_blocks) and decoded per device, rows
gathered with item_start rebased.  On a one-GPU box every shard goes to
cuda:0, which runs the same host code path; results must equal the oracle's
single-batch encode / decode bit for bit."""
import os
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "tests"))

pytestmark = pytest.mark.gpu

THREADS = min(16, os.cpu_count() or 1)


@pytest.mark.parametrize("shards", [1, 2, 3])
def test_encode_decode_sharded_match_oracle(gpu, shards):
    import pyoracle
    from helpers import counter_items
    lsmgpu = gpu
    items = counter_items(52 * 301, seed=11 + shards, tomb_frac=0.05)
    starts = pyoracle.cut_blocks(items, 4096)
    nb = len(starts) - 1
    bounds = lsmgpu.shard_items(starts, items.key_off, items.val_off, shards)
    assert bounds[0] == 0 and bounds[-1] == nb and all(a <= b for a, b in zip(bounds, bounds[1:]))
    ref_buf, ref_off = pyoracle.encode_blocks(items, starts, nthreads=THREADS)
    packed, block_off, status = lsmgpu.encode_sharded(items, starts, [0] * shards)
    assert (status == 0).all()
    assert (block_off == ref_off).all()
    assert packed.tobytes() == ref_buf.tobytes()
    parsed, item_start, st = pyoracle.decode_blocks(ref_buf, ref_off, nthreads=THREADS)
    res = lsmgpu.decode_sharded(packed, block_off, [0] * shards)
    assert (res["status"] == st).all() and (st == 0).all()
    assert (res["item_start"] == item_start.astype(np.int64)).all()
    n = int(item_start[-1])
    assert n == items.n
    for f, dt in (("seqno", np.uint64), ("key_off", np.uint32), ("val_off", np.uint32), ("val_len", np.uint32),
                  ("key_len", np.uint16), ("prefix_len", np.uint16), ("vtype", np.uint8)):
        assert (res[f].view(dt)[:n] == parsed[f].astype(dt)).all(), f


def test_decode_sharded_reports_per_block_status(gpu):
    """A corrupted block in the second shard keeps its own status at its global index."""
    import pyoracle
    from helpers import counter_items
    lsmgpu = gpu
    items = counter_items(52 * 64, seed=5)
    starts = pyoracle.cut_blocks(items, 4096)
    ref_buf, ref_off = pyoracle.encode_blocks(items, starts, nthreads=THREADS)
    bad = ref_buf.copy()
    b = len(ref_off) - 3
    bad[int(ref_off[b]) + 40] ^= 0x5A  # a payload byte: checksum mismatch
    parsed, item_start, st = pyoracle.decode_blocks(bad, ref_off, nthreads=THREADS)
    res = lsmgpu.decode_sharded(bad, ref_off, [0, 0])
    assert st[b] != 0 and (res["status"] == st).all()
