"""GPU parity of the batched point read (lsm_point_read_blocks) against the
oracle's DataBlock::point_read restatement (src/table/data_block/mod.rs:412-472):
hash-index probe (FREE / CONFLICT / bucket), restart binary search, MVCC scan.
Bar: identical hit index for every query, identical fields for every hit."""
import random

import numpy as np
import pytest

import pyoracle
from helpers import counter_items, index_items, pack, random_sorted_items

pytestmark = pytest.mark.gpu


def _run(gpu, buf, off, queries):
    """queries: list of (block, needle, snapshot) -> GPU result dict (numpy)."""
    import torch
    needles = b"".join(q[1] for q in queries)
    noff = np.zeros(len(queries) + 1, np.int64)
    noff[1:] = np.cumsum([len(q[1]) for q in queries])
    out = gpu.point_read(gpu.to_device_bytes(buf), torch.from_numpy(off.astype(np.int64)).cuda(), len(off) - 1,
                         torch.tensor([q[0] for q in queries], dtype=torch.int32).cuda(),
                         gpu.to_device_bytes(np.frombuffer(needles, np.uint8) if needles else np.zeros(0, np.uint8)),
                         torch.from_numpy(noff).cuda(),
                         torch.tensor([min(q[2], (1 << 63) - 1) for q in queries], dtype=torch.int64).cuda())
    torch.cuda.synchronize()
    return {k: v.cpu().numpy()[:len(queries)] for k, v in out.items()}


def _check(gpu, buf, off, queries):
    res = _run(gpu, buf, off, queries)
    parsed, item_start, status = pyoracle.decode_blocks(buf, off)
    assert (res["status"] == 0).all()
    hits = 0
    for q, (b, needle, snap) in enumerate(queries):
        payload = bytes(buf[int(off[b]) + 33:int(off[b + 1])])
        exp = pyoracle.point_read(payload, needle, min(snap, (1 << 63) - 1))
        assert int(res["item"][q]) == exp, (q, b, needle, snap)
        if exp >= 0:
            hits += 1
            r = int(item_start[b]) + exp
            assert int(res["seqno"][q]) == int(parsed["seqno"][r])
            assert int(res["val_off"][q]) == int(parsed["val_off"][r])
            assert int(res["val_len"][q]) == int(parsed["val_len"][r])
            assert int(res["vtype"][q]) == int(parsed["vtype"][r])
    return hits


@pytest.mark.parametrize("ri", [1, 2, 5, 16])
@pytest.mark.parametrize("ratio", [0.0, 1.33, 8.0])
def test_point_read_random_blocks(gpu, ri, ratio):
    rng = random.Random(ri * 31 + int(ratio * 10))
    # few distinct keys -> MVCC runs spanning restart intervals; vtypes incl. tombstones
    items = random_sorted_items(900, seed=ri + int(ratio * 7), kmin=1, kmax=6, alphabet=b"abc", vmax=40)
    starts = [0]
    while starts[-1] < items.n:
        starts.append(min(items.n, starts[-1] + rng.randint(1, 90)))
    starts = np.array(starts, np.uint32)
    buf, off = pyoracle.encode_blocks(items, starts, restart_interval=ri, hash_ratio=ratio)
    queries = []
    for b in range(len(starts) - 1):
        for i in range(int(starts[b]), int(starts[b + 1])):
            k = bytes(items.keys[int(items.key_off[i]):int(items.key_off[i + 1])])
            s = int(items.seqno[i])
            queries.append((b, k, s + 1))
            queries.append((b, k, rng.choice([0, 1, s, s + 2, 1 << 63])))
        for _ in range(6):  # misses and keys of other blocks
            other = rng.randrange(items.n)
            queries.append((b, bytes(items.keys[int(items.key_off[other]):int(items.key_off[other + 1])]),
                            rng.choice([1 << 63, 500])))
            queries.append((b, bytes(rng.choice(b"abcd") for _ in range(rng.randint(0, 7))), 1 << 63))
    hits = _check(gpu, buf, off, queries)
    assert hits > len(queries) // 4


def test_point_read_config2_shape(gpu):
    items = counter_items(52 * 512, seed=5)
    starts = pyoracle.cut_blocks(items, 4096)
    buf, off = pyoracle.encode_blocks(items, starts)
    rng = random.Random(9)
    queries = []
    for _ in range(4000):
        i = rng.randrange(items.n)
        b = int(np.searchsorted(starts, i, side="right")) - 1
        k = bytes(items.keys[int(items.key_off[i]):int(items.key_off[i + 1])])
        queries.append((b, k, rng.choice([64, 63, 1 << 63])))
    assert _check(gpu, buf, off, queries) > 1000


def test_point_read_status(gpu):
    items = counter_items(200, seed=2)
    starts = np.array([0, 100, 200], np.uint32)
    buf, off = pyoracle.encode_blocks(items, starts)
    ibuf, ioff = pyoracle.encode_blocks(index_items(50), np.array([0, 50], np.uint32), block_type=1)
    bad = bytearray(buf[int(off[1]):int(off[2])])
    bad[-31 + 2] ^= 0x7F  # trailer bin_len -> structural parse error
    blocks = [bytes(buf[:int(off[1])]), bytes(ibuf), bytes(bad)]
    pbuf, poff = pack(blocks)
    k = bytes(items.keys[:16])
    res = _run(gpu, pbuf, poff, [(0, k, 1 << 63), (1, k, 1 << 63), (2, k, 1 << 63)])
    assert list(res["status"]) == [0, 7, 5]
    assert int(res["item"][0]) == 0 and int(res["item"][1]) == -1 and int(res["item"][2]) == -1
