"""Compact decode output (lsm_decode_blocks16, lsm_parsed_items16): the same
walk as lsm_decode_blocks (decoder.rs:442-483, data_block/mod.rs:272-316) with
16-bit payload offsets and lengths, 19 B/item.  Oracle: pyoracle.decode_blocks
(the 32-bit layout) narrowed to 16 bits, plus the compact rule: a block the
oracle would parse (status OK, PARSE or OVERFLOW, i.e. past the header,
checksum, data_length and type checks) that is an index block or has a payload
over 65535 bytes gets LSM_UNSUPPORTED.  Bar: bit-exact statuses, item_start and
every field of every OK block."""
import numpy as np
import pytest

import pyoracle
from helpers import counter_items, index_items, pack, prefix_items, random_sorted_items

pytestmark = pytest.mark.gpu

FIELD16 = {"seqno": np.uint64, "key_off": np.uint16, "val_off": np.uint16, "val_len": np.uint16,
           "key_len": np.uint16, "prefix_len": np.uint16, "vtype": np.uint8}
UNSUPPORTED = 9


def _compact_expected(buf, off, status):
    exp = status.copy()
    for b in range(len(off) - 1):
        blk = bytes(buf[int(off[b]):int(off[b + 1])])
        st, h = pyoracle.header_decode(blk)
        if status[b] in (0, 5, 6) and (h.block_type == 1 or len(blk) - 33 > 0xFFFF):
            exp[b] = UNSUPPORTED
    return exp


def _gpu_decode16(gpu, buf, off, tuning=None):
    import torch
    d_blocks = gpu.to_device_bytes(buf)
    d_off = torch.from_numpy(off.astype(np.int64)).cuda()
    n = len(off) - 1
    out = gpu.decode_blocks(d_blocks, d_off, n, item_cap=len(buf) // 3 + 1, tuning=tuning, compact=True)
    torch.cuda.synchronize()
    res = {k: v.cpu().numpy() for k, v in out.items()}
    res["status"] = res["status"][:n]
    return res


def _check(gpu, buf, off, tuning=None):
    parsed, item_start, status = pyoracle.decode_blocks(buf, off)
    g = _gpu_decode16(gpu, buf, off, tuning)
    exp = _compact_expected(buf, off, status)
    st = g["status"].astype(np.int32)
    assert (st == exp).all(), (np.nonzero(st != exp)[0][:10], st[:10], exp[:10])
    assert (g["item_start"].view(np.uint32) == item_start).all()
    ok = np.nonzero(exp == 0)[0]
    starts = item_start.astype(np.int64)
    mask = np.zeros(int(starts[-1]), bool)
    for b in ok:
        mask[starts[b]:starts[b + 1]] = True
    for f, dt in FIELD16.items():
        o = parsed[f][:len(mask)]
        assert (o[mask] <= np.iinfo(dt).max).all(), f
        gv = g[f].view(dt)[:len(mask)]
        bad = np.nonzero((gv != o.astype(dt)) & mask)[0]
        assert len(bad) == 0, (f, bad[:10], gv[bad[:10]], o[bad[:10]])
    return exp


@pytest.mark.parametrize("shape", ["counter4k", "prefix16k", "random"])
def test_compact_matches_oracle(gpu, shape):
    if shape == "counter4k":
        items = counter_items(60000, seed=3, tomb_frac=0.02)
        starts = pyoracle.cut_blocks(items, 4096)
    elif shape == "prefix16k":
        items = prefix_items(20000)
        starts = pyoracle.cut_blocks(items, 16384)
    else:
        items = random_sorted_items(6000, seed=5, kmax=60, vmax=300)
        starts = pyoracle.cut_blocks(items, 4096)
    buf, off = pyoracle.encode_blocks(items, starts, hash_ratio=0.75 if shape == "random" else 0.0)
    exp = _check(gpu, buf, off)
    assert (exp == 0).all()


def test_compact_big_index_and_corrupt_blocks(gpu):
    """Every route: group kernel (4 KiB blocks, index blocks -> UNSUPPORTED),
    big-block kernel (57 KB payloads that still fit), general path (a 78 KB
    payload -> UNSUPPORTED), and a checksum error on each side of the size rule."""
    small = counter_items(3000, seed=11)
    b4, o4 = pyoracle.encode_blocks(small, pyoracle.cut_blocks(small, 4096))
    blocks = [bytes(b4[int(o4[i]):int(o4[i + 1])]) for i in range(len(o4) - 1)]
    big = counter_items(2400, seed=12)
    bb, ob = pyoracle.encode_blocks(big, np.array([0, 800, 1600, 2400], np.uint32))  # ~64 KiB payloads
    bigs = [bytes(bb[int(ob[i]):int(ob[i + 1])]) for i in range(3)]
    assert all(32 * 1024 < len(x) - 33 <= 0xFFFF for x in bigs), [len(x) for x in bigs]
    huge = counter_items(1200, seed=13)
    bh, oh = pyoracle.encode_blocks(huge, np.array([0, 1100, 1200], np.uint32))  # ~78 KB payload
    assert int(oh[1]) - 33 > 0xFFFF
    idx = index_items(400)
    bi, oi = pyoracle.encode_blocks(idx, np.array([0, 200, 400], np.uint32), block_type=1)
    bad_ck = bytearray(blocks[1])
    bad_ck[200] ^= 1  # payload checksum: CKSUM before the compact rule
    bad_hdr = bytearray(bytes(bh[:int(oh[1])]))
    bad_hdr[40] ^= 1  # a >64 KiB payload with a bad checksum still reports CKSUM
    tests = (blocks[:5] + bigs + [bytes(bh[:int(oh[1])]), bytes(bi[:int(oi[1])])] + blocks[5:9] +
             [bytes(bad_ck), bytes(bad_hdr), bytes(bi[int(oi[1]):int(oi[2])])] + blocks[9:])
    buf, off = pack(tests)
    exp = _check(gpu, buf, off)
    assert (exp == UNSUPPORTED).sum() == 3 and (exp == 4).sum() == 2, exp


def test_compact_config1_slice_against_full_layout(gpu):
    """A configs[1]-shaped batch: the compact fields equal the 32-bit decode's."""
    import torch
    items = counter_items(200000, seed=21)
    starts = pyoracle.cut_blocks(items, 4096)
    buf, off = pyoracle.encode_blocks(items, starts)
    d_blocks = gpu.to_device_bytes(buf)
    d_off = torch.from_numpy(off.astype(np.int64)).cuda()
    n = len(off) - 1
    full = gpu.decode_blocks(d_blocks, d_off, n, item_cap=items.n)
    comp = gpu.decode_blocks(d_blocks, d_off, n, item_cap=items.n, compact=True)
    torch.cuda.synchronize()
    assert int((full["status"][:n] != 0).sum()) == 0 and int((comp["status"][:n] != 0).sum()) == 0
    assert torch.equal(full["item_start"], comp["item_start"])
    for f in ("key_off", "val_off", "val_len"):
        a, b = full[f][:items.n].to(torch.int64), comp[f][:items.n].to(torch.int64) & 0xFFFF
        assert int(a.max()) <= 0xFFFF and torch.equal(a, b), f
    for f in ("seqno", "key_len", "prefix_len", "vtype"):
        assert torch.equal(full[f][:items.n], comp[f][:items.n]), f
