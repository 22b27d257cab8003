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


def test_threaded_shards_index_and_random_keys(gpu):
    """Four shard threads at once on cuda:0 (the host path of a 4-GPU run: one
    thread, stream and pinned staging per shard, the exchange step behind a
    barrier): random sorted keys with tombstones, then the index blocks of those
    data blocks; encode bytes and decoded rows equal the oracle's."""
    import pyoracle
    from helpers import random_sorted_items
    lsmgpu = gpu
    items = random_sorted_items(52 * 700, seed=29)
    starts = pyoracle.cut_blocks(items, 4096)
    ref_buf, ref_off = pyoracle.encode_blocks(items, starts, nthreads=THREADS)
    packed, block_off, status = lsmgpu.encode_sharded(items, starts, [0, 0, 0, 0])
    assert (status == 0).all() and (block_off == ref_off).all() and packed.tobytes() == ref_buf.tobytes()
    # index blocks over those data blocks: (last key, seqno, handle) per block, 100 handles per index block
    nb = len(starts) - 1
    last = starts[1:].astype(np.int64) - 1
    keys = [bytes(items.keys[int(items.key_off[i]):int(items.key_off[i + 1])]) for i in last]
    kl = np.array([len(k) for k in keys], np.uint64)
    ix = pyoracle.Items(np.frombuffer(b"".join(keys), np.uint8), np.concatenate([[0], np.cumsum(kl)]).astype(np.uint64),
                        np.zeros(1, np.uint8), np.zeros(nb + 1, np.uint64), items.seqno[last], np.zeros(nb, np.uint8),
                        ref_off[:nb].astype(np.uint64), (ref_off[1:] - ref_off[:nb]).astype(np.uint32))
    istarts = np.array(list(range(0, nb, 100)) + [nb], np.uint32)
    iref_buf, iref_off = pyoracle.encode_blocks(ix, istarts, restart_interval=1, block_type=1, nthreads=THREADS)
    ipacked, ioff, ist = lsmgpu.encode_sharded(ix, istarts, [0, 0, 0], restart_interval=1,
                                               block_type=lsmgpu.BLOCK_INDEX)
    assert (ist == 0).all() and (ioff == iref_off).all() and ipacked.tobytes() == iref_buf.tobytes()
    parsed, item_start, st = pyoracle.decode_blocks(iref_buf, iref_off, nthreads=THREADS)
    res = lsmgpu.decode_sharded(ipacked, ioff, [0, 0, 0])
    assert (res["status"] == st).all() and (st == 0).all()
    n = int(item_start[-1])
    assert n == nb and (res["item_start"] == item_start.astype(np.int64)).all()
    assert (res["handle_off"].view(np.uint64)[:n] == parsed["handle_off"].astype(np.uint64)).all()
    assert (res["val_len"].view(np.uint32)[:n] == parsed["val_len"].astype(np.uint32)).all()
