"""Shared test helpers: synthetic item batches (BASELINE.md generators) and
GPU-vs-oracle comparisons."""
from __future__ import annotations

import random

import numpy as np

import pyoracle


def splitmix64(seed):
    """BASELINE.md seed stream: splitmix64(0x5EED_0001 + cfg)."""
    x = seed & 0xFFFFFFFFFFFFFFFF
    while True:
        x = (x + 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF
        z = x
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
        yield z ^ (z >> 31)


def counter_items(n, key_len=16, val_len=64, seqno=63, seed=1, start=0, tomb_frac=0.0):
    """Config 1/2 shape: keys = big-endian counter (key_len bytes), random values."""
    rng = np.random.default_rng(seed)
    ctr = np.arange(start, start + n, dtype=np.uint64)
    keys = np.zeros((n, key_len), np.uint8)
    for b in range(min(8, key_len)):
        keys[:, key_len - 1 - b] = ((ctr >> np.uint64(8 * b)) & np.uint64(0xFF)).astype(np.uint8)
    vtype = np.zeros(n, np.uint8)
    if tomb_frac > 0:
        vtype[rng.random(n) < tomb_frac] = 1
    vlens = np.where(vtype == 1, 0, val_len).astype(np.uint64)
    vals = rng.integers(0, 256, int(vlens.sum()), dtype=np.uint8)
    key_off = np.arange(n + 1, dtype=np.uint64) * np.uint64(key_len)
    val_off = np.concatenate([[0], np.cumsum(vlens)]).astype(np.uint64)
    seq = np.full(n, seqno, np.uint64)
    return pyoracle.Items(keys.reshape(-1), key_off, vals, val_off, seq, vtype)


def prefix_items(n, prefix_len=32, suffix_len=8, val_len=256, seed=4):
    """Config 4 shape: fixed random 32 B prefix || 8 B BE counter, 256 B values."""
    rng = np.random.default_rng(seed)
    pre = rng.integers(0, 256, prefix_len, dtype=np.uint8)
    ctr = np.arange(n, dtype=np.uint64)
    suf = np.zeros((n, suffix_len), np.uint8)
    for b in range(suffix_len):
        suf[:, suffix_len - 1 - b] = ((ctr >> np.uint64(8 * b)) & np.uint64(0xFF)).astype(np.uint8)
    keys = np.concatenate([np.tile(pre, (n, 1)), suf], axis=1).reshape(-1)
    kl = prefix_len + suffix_len
    vals = rng.integers(0, 256, n * val_len, dtype=np.uint8)
    return pyoracle.Items(keys, np.arange(n + 1, dtype=np.uint64) * np.uint64(kl), vals,
                          np.arange(n + 1, dtype=np.uint64) * np.uint64(val_len), np.full(n, 63, np.uint64),
                          np.zeros(n, np.uint8))


def random_sorted_items(n, seed=0, kmin=1, kmax=24, vmax=80, alphabet=b"abcdefg", big_seq=False,
                        vtypes=(0, 1, 2, 4)):
    rng = random.Random(seed)
    raw = {}
    while len(raw) < n:
        k = bytes(rng.choice(alphabet) for _ in range(rng.randint(kmin, kmax)))
        s = rng.getrandbits(63) if big_seq else rng.randint(0, 1000)
        t = rng.choice(vtypes)
        v = b"" if t in (1, 2) else bytes(rng.getrandbits(8) for _ in range(rng.randint(0, vmax)))
        raw[(k, s)] = (v, t)
    keys = sorted(raw, key=lambda ks: (ks[0], -ks[1]))
    return pyoracle.Items.from_list([(k, raw[(k, s)][0], s, raw[(k, s)][1]) for k, s in keys])


def index_items(n, seed=9):
    rng = random.Random(seed)
    keys = b"".join(b"end-key-%08d" % (3 * i) for i in range(n))
    kl = np.full(n, 16, np.uint64)
    key_off = np.concatenate([[0], np.cumsum(kl)]).astype(np.uint64)
    sizes = np.array([rng.randint(100, 70000) for _ in range(n)], np.uint32)
    offs = np.concatenate([[0], np.cumsum(sizes.astype(np.uint64))[:-1]]).astype(np.uint64)
    seq = np.array([rng.getrandbits(63) for _ in range(n)], np.uint64)
    return pyoracle.Items(np.frombuffer(keys, np.uint8), key_off, np.zeros(1, np.uint8), np.zeros(n + 1, np.uint64),
                          seq, np.zeros(n, np.uint8), offs, sizes)


def pack(blocks: list[bytes]):
    """List of on-disk blocks -> (contiguous uint8 array, uint64 offsets)."""
    off = np.zeros(len(blocks) + 1, np.uint64)
    off[1:] = np.cumsum([len(b) for b in blocks])
    return np.frombuffer(b"".join(blocks), np.uint8).copy(), off


def gpu_decode(L, blocks_np, off_np, expect_type=-1, tuning=None, item_cap=None, pool=True, workspace_bytes=None,
               compact=False):
    import torch
    d_blocks = L.to_device_bytes(blocks_np)
    d_off = torch.from_numpy(off_np.astype(np.int64)).cuda()
    n = len(off_np) - 1
    item_cap = item_cap if item_cap is not None else len(blocks_np) // 3 + 1
    out = L.decode_blocks(d_blocks, d_off, n, expect_type=expect_type, item_cap=item_cap, tuning=tuning, pool=pool,
                          workspace_bytes=workspace_bytes, compact=compact)
    torch.cuda.synchronize()
    res = {k: v.cpu().numpy() for k, v in out.items()}
    res["status"] = res["status"][:n]
    return res


FIELD_VIEW = {"seqno": np.uint64, "key_off": np.uint32, "val_off": np.uint32, "val_len": np.uint32,
              "key_len": np.uint16, "prefix_len": np.uint16, "vtype": np.uint8, "handle_off": np.uint64}


def compare_decode(gpu, ora_parsed, ora_item_start, ora_status):
    """GPU decode result == oracle decode result (status for all blocks; every
    parsed field for OK blocks)."""
    st_g = gpu["status"].astype(np.int32)
    assert (st_g == ora_status).all(), (np.nonzero(st_g != ora_status)[0][:10], st_g[:10], ora_status[:10])
    assert (gpu["item_start"].view(np.uint32) == ora_item_start).all()
    ok = np.nonzero(ora_status == 0)[0]
    if len(ok) == 0:
        return
    starts = ora_item_start.astype(np.int64)
    mask = np.zeros(int(starts[-1]), bool)
    for b in ok:
        mask[starts[b]:starts[b + 1]] = True
    for f, dt in FIELD_VIEW.items():
        g = gpu[f].view(dt)[:len(mask)]
        o = ora_parsed[f][:len(mask)].astype(dt)
        bad = np.nonzero((g != o) & mask)[0]
        assert len(bad) == 0, (f, bad[:10], g[bad[:10]], o[bad[:10]])
