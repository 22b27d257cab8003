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


def test_point_read_corrupt_hash_index(gpu):
    """Blocks whose hash index (bucket bytes, or the trailer's hash_len / hash_off)
    is corrupted and re-sealed with a valid checksum: a bucket naming a restart
    interval the block does not have, or a bucket region past the trailer, is
    PARSE (the reference would index out of range and panic); any other bucket
    value sends the scan to that interval, as the reference's seek does.  GPU
    status and hit index equal the oracle's (-2 = its parse error)."""
    rng = random.Random(77)
    items = random_sorted_items(400, seed=3, kmin=2, kmax=8, vmax=30)
    starts = np.array(list(range(0, 400, 40)) + [400], np.uint32)
    blocks, queries = [], []
    for b in range(len(starts) - 1):
        one = pyoracle.Items(items.keys, items.key_off, items.vals, items.val_off, items.seqno, items.vtype)
        payload = bytearray(pyoracle.data_block_encode(one, int(starts[b]), 40, restart_interval=4, hash_ratio=1.5))
        tr = len(payload) - 31
        hash_len = int.from_bytes(payload[tr + 10:tr + 14], "little")
        hash_off = int.from_bytes(payload[tr + 14:tr + 18], "little")
        assert hash_len > 0
        kind = b % 4
        if kind == 0:    # buckets -> restart indexes beyond bin_len, or other valid ones
            for _ in range(hash_len // 2):
                payload[hash_off + rng.randrange(hash_len)] = rng.choice([11, 12, 50, 200, 0, 1, 5])
        elif kind == 1:  # bucket region runs into the trailer
            payload[tr + 10:tr + 14] = (hash_len + rng.randint(1, 40)).to_bytes(4, "little")
        elif kind == 2:  # hash_off moved
            payload[tr + 14:tr + 18] = (hash_off + rng.choice([-3, 5, 1000])).to_bytes(4, "little", signed=True)
        blocks.append(pyoracle.block_write(bytes(payload)))
        for i in range(int(starts[b]), int(starts[b + 1])):
            k = bytes(items.keys[int(items.key_off[i]):int(items.key_off[i + 1])])
            queries.append((b, k, 1 << 63))
    buf, off = pack(blocks)
    res = _run(gpu, buf, off, queries)
    for q, (b, needle, snap) in enumerate(queries):
        payload = bytes(buf[int(off[b]) + 33:int(off[b + 1])])
        exp = pyoracle.point_read(payload, needle, (1 << 63) - 1)
        if exp == -2:
            assert int(res["status"][q]) == 5, (q, b)
        else:
            assert int(res["status"][q]) == 0 and int(res["item"][q]) == exp, (q, b, exp, int(res["item"][q]))


@pytest.mark.parametrize("ri", [1, 3, 16])
def test_seek_random_bounds(gpu, ri):
    """lsm_seek_blocks vs the oracle's Iter::seek / seek_upper restatement on random
    MVCC blocks (few distinct keys, so equal keys span restart intervals), random
    bounds (present keys, absent keys, empty needles) and every flag combination
    including the exclusive forms (data_block/iter.rs:37-176)."""
    import torch
    rng = random.Random(ri)
    items = random_sorted_items(700, seed=50 + ri, kmin=1, kmax=5, alphabet=b"abcd", vmax=20)
    starts = [0]
    while starts[-1] < items.n:
        starts.append(min(items.n, starts[-1] + rng.randint(1, 70)))
    starts = np.array(starts, np.uint32)
    buf, off = pyoracle.encode_blocks(items, starts, restart_interval=ri, hash_ratio=rng.choice([0.0, 1.33]))
    qs = []
    for _ in range(3000):
        b = rng.randrange(len(starts) - 1)

        def bound():
            if rng.random() < 0.6:
                i = rng.randrange(items.n)
                return bytes(items.keys[int(items.key_off[i]):int(items.key_off[i + 1])])
            return bytes(rng.choice(b"abcde") for _ in range(rng.randint(0, 5)))
        qs.append((b, bound(), bound(), rng.randrange(16)))
    lo, loff = np.frombuffer(b"".join(q[1] for q in qs) or b"\0", np.uint8), np.zeros(len(qs) + 1, np.int64)
    loff[1:] = np.cumsum([len(q[1]) for q in qs])
    hi, hoff = np.frombuffer(b"".join(q[2] for q in qs) or b"\0", np.uint8), np.zeros(len(qs) + 1, np.int64)
    hoff[1:] = np.cumsum([len(q[2]) for q in qs])
    res = gpu.seek(gpu.to_device_bytes(buf), torch.from_numpy(off.astype(np.int64)).cuda(), len(starts) - 1,
                   torch.tensor([q[0] for q in qs], dtype=torch.int32).cuda(), gpu.to_device_bytes(lo),
                   torch.from_numpy(loff).cuda(), gpu.to_device_bytes(hi), torch.from_numpy(hoff).cuda(),
                   torch.tensor([q[3] for q in qs], dtype=torch.uint8).cuda())
    torch.cuda.synchronize()
    res = {k: v.cpu().numpy() for k, v in res.items()}
    assert (res["status"][:len(qs)] == 0).all()
    for q, (b, lb, hb, fl) in enumerate(qs):
        payload = bytes(buf[int(off[b]) + 33:int(off[b + 1])])
        exp = pyoracle.seek(payload, lb if fl & 1 else None, hb if fl & 2 else None, bool(fl & 4), bool(fl & 8))
        got = (int(res["first"][q]), int(res["end"][q]), bool(res["found"][q] & 1), bool(res["found"][q] & 2))
        assert got == exp, (q, b, lb, hb, fl, got, exp)
