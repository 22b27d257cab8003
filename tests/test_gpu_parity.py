"""GPU parity tests: the HIP product path (through the C ABI) against the oracle
and the committed golden vectors.  Bar: bit-exact bytes / fields / statuses.
"""
import random

import numpy as np
import pytest

import pyoracle
from conftest import case_expected_items, case_items
from helpers import (FIELD_VIEW, compare_decode, counter_items, gpu_decode, index_items, pack, prefix_items,
                     random_sorted_items)

pytestmark = pytest.mark.gpu


def _torch():
    import torch
    return torch


# ------------------------------------------------------------------ XXH3

def test_xxh3_batch_kats(gpu, xxh3_kat):
    torch = _torch()
    chunks, off = [], [0]
    rng = random.Random(1)
    pad_first = []
    for v in xxh3_kat:
        n = v["len"]
        lead = rng.randint(0, 17)  # every alignment of the range start
        b = bytes(rng.getrandbits(8) for _ in range(lead)) + bytes(((31 * i + 7) & 0xFF) for i in range(n))
        chunks.append(b)
        pad_first.append(lead)
    data = b"".join(chunks)
    starts, ends = [], []
    pos = 0
    for lead, c in zip(pad_first, chunks):
        starts.append(pos + lead)
        ends.append(pos + len(c))
        pos += len(c)
    # ranges are disjoint but not contiguous: encode each as its own [start,end) via two-entry offsets
    d = gpu.to_device_bytes(data)
    res = []
    for s, e in zip(starts, ends):
        off_t = torch.tensor([s, e], dtype=torch.int64, device="cuda")
        res.append(gpu.xxh3_128_batch(d, off_t, 1))
    torch.cuda.synchronize()
    for v, r in zip(xxh3_kat, res):
        lo, hi = [int(x) & 0xFFFFFFFFFFFFFFFF for x in r.cpu().tolist()[:2]]
        assert (hi << 64) | lo == int(v["xxh3_128"]), v["len"]


def test_xxh3_batch_random(gpu):
    torch = _torch()
    rng = np.random.default_rng(2)
    data = rng.integers(0, 256, 300000, dtype=np.uint8)
    cuts = np.sort(rng.choice(np.arange(1, len(data)), 200, replace=False))
    off = np.concatenate([[0], cuts, [len(data)]]).astype(np.int64)
    d = gpu.to_device_bytes(data)
    out = gpu.xxh3_128_batch(d, torch.from_numpy(off).cuda(), len(off) - 1).cpu().numpy().view(np.uint64)
    for i in range(len(off) - 1):
        exp = pyoracle.xxh3_128(data[off[i]:off[i + 1]].tobytes())
        assert (int(out[2 * i + 1]) << 64) | int(out[2 * i]) == exp, i


# ------------------------------------------------------------------ golden

def test_decode_golden_blocks(gpu, golden_blocks):
    blocks = [bytes.fromhex(c["block"]) for c in golden_blocks]
    buf, off = pack(blocks)
    g = gpu_decode(gpu, buf, off)
    parsed, item_start, status = pyoracle.decode_blocks(buf, off)
    assert (status == 0).all()
    compare_decode(g, parsed, item_start, status)
    # and materialised items equal the golden inputs
    for b, case in enumerate(golden_blocks):
        s0, s1 = int(item_start[b]), int(item_start[b + 1])
        payload = blocks[b][33:]
        one = {f: g[f].view(dt)[s0:s1] for f, dt in FIELD_VIEW.items()}
        if case["kind"] == "index":
            for j, (k, s, o, sz) in enumerate(case_expected_items(case)):
                ko, kl = int(one["key_off"][j]), int(one["key_len"][j])
                assert payload[ko:ko + kl] == k and int(one["seqno"][j]) == s
                assert int(one["handle_off"][j]) == o and int(one["val_len"][j]) == sz
        else:
            assert pyoracle.materialize(payload, one, case["restart_interval"]) == case_expected_items(case), case["name"]


# (blocks_per_wave, stage bytes, tile items[, flags])
TUNINGS = [None,                                 # library defaults
           (48, 65536, 1024), (1, 256, 64),      # 64 KiB stage; every block larger than the stage: general path
           (63, 65536, 2048), (5, 4096, 64), (3, 8192, 128), (8, 32768, 512)]


@pytest.mark.parametrize("tuning", TUNINGS)
def test_decode_golden_blocks_tunings(gpu, golden_blocks, tuning):
    """The group kernel under several stage / group shapes and the general path
    (tiny stages) all agree with the oracle."""
    blocks = [bytes.fromhex(c["block"]) for c in golden_blocks]
    buf, off = pack(blocks)
    g = gpu_decode(gpu, buf, off, tuning=tuning)
    parsed, item_start, status = pyoracle.decode_blocks(buf, off)
    compare_decode(g, parsed, item_start, status)


def _gpu_encode(gpu, items, starts, ri, ratio, block_type):
    torch = _torch()
    d_items = gpu.items_to_device(items)
    d_starts = torch.from_numpy(np.asarray(starts, np.int64).astype(np.int32)).cuda()
    out = gpu.Encoder().encode(d_items, d_starts, len(starts) - 1, restart_interval=ri, hash_ratio=ratio,
                               block_type=block_type)
    torch.cuda.synchronize()
    off = out["block_off"].cpu().numpy().view(np.uint64)
    buf = out["buf"].cpu().numpy()[:int(off[-1])]
    return buf, off, out["status"].cpu().numpy()[:len(starts) - 1]


def test_encode_golden_blocks(gpu, golden_blocks):
    for case in golden_blocks:
        items = case_items(case)
        buf, off, st = _gpu_encode(gpu, items, [0, items.n], case["restart_interval"], case["hash_ratio"],
                                   case["block_type"])
        assert (st == 0).all(), case["name"]
        assert buf.tobytes().hex() == case["block"], case["name"]


# ------------------------------------------------------------------ fuzz-like

@pytest.mark.parametrize("ri", [1, 2, 5, 16, 64])
@pytest.mark.parametrize("ratio", [0.0, 1.33])
def test_encode_decode_random_batches(gpu, ri, ratio):
    items = random_sorted_items(3000, seed=ri * 7 + int(ratio), vmax=120)
    rng = random.Random(ri)
    # random cut points (blocks of 1..120 items)
    starts = [0]
    while starts[-1] < items.n:
        starts.append(min(items.n, starts[-1] + rng.randint(1, 120)))
    starts = np.array(starts, np.uint32)
    ref_buf, ref_off = pyoracle.encode_blocks(items, starts, restart_interval=ri, hash_ratio=ratio)
    buf, off, st = _gpu_encode(gpu, items, starts, ri, ratio, 0)
    assert (st == 0).all()
    assert (off == ref_off).all()
    assert buf.tobytes() == ref_buf.tobytes()
    g = gpu_decode(gpu, buf, off)
    parsed, item_start, status = pyoracle.decode_blocks(buf, off)
    assert (status == 0).all()
    compare_decode(g, parsed, item_start, status)


def test_hash_index_key_lengths(gpu):
    """Hash-index buckets of keys of 0..300 bytes: the plan pass hashes keys of
    <= 16 bytes from their first 16 bytes and leaves longer ones (every XXH3
    length class, up to the > 240-byte long path) to encode_bucket_fixup_kernel;
    bit-exact against the oracle."""
    for kmin, kmax, seed in ((1, 16, 11), (17, 300, 12), (1, 300, 13)):
        items = random_sorted_items(2000, seed=seed, kmin=kmin, kmax=kmax, vmax=40)
        rng = random.Random(seed)
        starts = [0]
        while starts[-1] < items.n:
            starts.append(min(items.n, starts[-1] + rng.randint(8, 40)))
        starts = np.array(starts, np.uint32)
        ref_buf, ref_off = pyoracle.encode_blocks(items, starts, restart_interval=4, hash_ratio=1.33)
        buf, off, st = _gpu_encode(gpu, items, starts, 4, 1.33, 0)
        assert (st == 0).all()
        assert (off == ref_off).all()
        assert buf.tobytes() == ref_buf.tobytes(), (kmin, kmax)


@pytest.mark.parametrize("ratio", [0.0, 1.33])
def test_encode_size_classes(gpu, ratio):
    """Blocks in every encode class (LDS image <= 5 KiB, <= 20 KiB, <= 96 KiB,
    HBM-direct beyond) with unaligned key/value arena offsets and long values,
    bit-exact against the oracle."""
    items = random_sorted_items(1500, seed=int(ratio * 100) + 5, kmax=40, vmax=700, big_seq=True)
    rng = random.Random(77)
    starts = [0]
    for want in (3, 40, 9, 150, 1, 400, 25, 60, 700, 2, 110):  # ~0.3 .. 250 KiB blocks
        starts.append(min(items.n, starts[-1] + want))
    while starts[-1] < items.n:
        starts.append(min(items.n, starts[-1] + rng.randint(1, 300)))
    starts = np.array(starts, np.uint32)
    ref_buf, ref_off = pyoracle.encode_blocks(items, starts, restart_interval=16, hash_ratio=ratio)
    sizes = np.diff(ref_off.astype(np.int64))
    assert sizes.max() > 100 * 1024 and sizes.min() < 4096
    buf, off, st = _gpu_encode(gpu, items, starts, 16, ratio, 0)
    assert (st == 0).all()
    assert (off == ref_off).all()
    assert buf.tobytes() == ref_buf.tobytes()


def test_index_blocks(gpu):
    items = index_items(2000)
    starts = np.array(list(range(0, 2000, 97)) + [2000], np.uint32)
    ref_buf, ref_off = pyoracle.encode_blocks(items, starts, block_type=1)
    buf, off, st = _gpu_encode(gpu, items, starts, 1, 0.0, 1)
    assert (st == 0).all() and buf.tobytes() == ref_buf.tobytes()
    for et in (-1, 1):
        g = gpu_decode(gpu, buf, off, expect_type=et)
        parsed, item_start, status = pyoracle.decode_blocks(buf, off, expect_type=et)
        assert (status == 0).all()
        compare_decode(g, parsed, item_start, status)
    g = gpu_decode(gpu, buf, off, expect_type=0)
    assert (g["status"] == 7).all()  # TYPE_MISMATCH (util.rs:81-86)


def test_large_index_blocks(gpu):
    """Full block indexes larger than the general path's stage (> 72 KiB, as a
    64 MiB table of 4 KiB blocks has): decoded through the stage in 64 KiB
    chunks with the XXH3 chain carried across them (decode_index_chunked).
    Valid blocks, a flipped payload bit (CKSUM), a broken record re-sealed with
    valid checksums, and a re-sealed item count that leaves the last interval
    two records (the interval walk fallback): statuses and fields == oracle."""
    items = index_items(14000, seed=11)
    starts = np.array([0, 6000, 6001, 14000], np.uint32)
    buf, off = pyoracle.encode_blocks(items, starts, block_type=1)
    assert np.diff(off.astype(np.int64)).max() > 150 * 1024
    blocks = [bytes(buf[int(off[i]):int(off[i + 1])]) for i in range(3)]
    bad_ck = bytearray(blocks[0])
    bad_ck[33 + 70000] ^= 0x10
    rec = bytearray(blocks[2][33:])
    step, bin_off = rec[-30], int.from_bytes(rec[-25:-21], "little")  # trailer.rs:118-163
    start = int.from_bytes(rec[bin_off + step * 4000:bin_off + step * 4001], "little")
    rec[start] = 1  # record 4000's tag byte (index records start with 0)
    cnt = bytearray(blocks[2][33:])
    cnt[-4] += 1  # item_count = bin_len + 1
    tests = blocks + [bytes(bad_ck), pyoracle.block_write(bytes(rec), 1), pyoracle.block_write(bytes(cnt), 1)]
    buf2, off2 = pack(tests)
    g = gpu_decode(gpu, buf2, off2)
    parsed, item_start, status = pyoracle.decode_blocks(buf2, off2)
    assert (status[:3] == 0).all() and status[3] == 4 and (status[4:] != 0).all(), status
    compare_decode(g, parsed, item_start, status)


# ------------------------------------------------------------------ configs (reduced counts)

def test_config2_shape_counter_keys(gpu):
    items = counter_items(52 * 2048, seed=21)
    starts = pyoracle.cut_blocks(items, 4096)
    assert len(starts) - 1 == 2048
    ref_buf, ref_off = pyoracle.encode_blocks(items, starts)
    buf, off, st = _gpu_encode(gpu, items, starts, 16, 0.0, 0)
    assert (st == 0).all() and buf.tobytes() == ref_buf.tobytes()
    g = gpu_decode(gpu, buf, off)
    parsed, item_start, status = pyoracle.decode_blocks(buf, off)
    compare_decode(g, parsed, item_start, status)


def test_config4_prefix_heavy_16k(gpu):
    items = prefix_items(56 * 300)
    starts = pyoracle.cut_blocks(items, 16384)
    ref_buf, ref_off = pyoracle.encode_blocks(items, starts)
    assert int(ref_off[1]) == 14953
    buf, off, st = _gpu_encode(gpu, items, starts, 16, 0.0, 0)
    assert (st == 0).all() and buf.tobytes() == ref_buf.tobytes()
    for tuning in (None, (8, 32768, 512)):
        g = gpu_decode(gpu, buf, off, tuning=tuning)
        parsed, item_start, status = pyoracle.decode_blocks(buf, off)
        compare_decode(g, parsed, item_start, status)


def test_64k_blocks_u32_binary_index(gpu):
    """64 KiB random-key blocks: binary-index step 4 (builder.rs:22-32), larger
    than the default LDS stage -> the direct-from-HBM paths."""
    rng = np.random.default_rng(8)
    n = 820 * 12
    keys = np.sort(rng.integers(0, 2 ** 63, n, dtype=np.uint64))
    import pyoracle as po
    kb = keys.byteswap().view(np.uint8).reshape(n, 8)
    keys16 = np.concatenate([kb, rng.integers(0, 256, (n, 8), dtype=np.uint8)], axis=1).reshape(-1)
    vals = rng.integers(0, 256, n * 64, dtype=np.uint8)
    items = po.Items(keys16, np.arange(n + 1, dtype=np.uint64) * np.uint64(16), vals,
                     np.arange(n + 1, dtype=np.uint64) * np.uint64(64), np.full(n, 63, np.uint64), np.zeros(n, np.uint8))
    starts = po.cut_blocks(items, 65536)
    ref_buf, ref_off = po.encode_blocks(items, starts)
    p0 = ref_buf[33:int(ref_off[1])].tobytes()
    assert p0[-31 + 1] == 4  # u32 binary index
    buf, off, st = _gpu_encode(gpu, items, starts, 16, 0.0, 0)
    assert (st == 0).all() and buf.tobytes() == ref_buf.tobytes()
    g = gpu_decode(gpu, buf, off)
    parsed, item_start, status = po.decode_blocks(buf, off)
    compare_decode(g, parsed, item_start, status)


# ------------------------------------------------------------------ corruption / edge cases

def test_corruption_statuses_match_oracle(gpu):
    items = random_sorted_items(2500, seed=5)
    starts = np.array(list(range(0, 2500, 50)) + [2500], np.uint32)
    buf, off = pyoracle.encode_blocks(items, starts, restart_interval=4, hash_ratio=1.0)
    buf = buf.copy()
    rng = random.Random(99)
    nb = len(off) - 1
    for b in range(0, nb, 2):
        o, e = int(off[b]), int(off[b + 1])
        where = rng.choice(["magic", "type", "hdr", "payload", "trailer", "len"])
        if where == "magic":
            buf[o] ^= 0x40
        elif where == "type":
            buf[o + 4] = rng.choice([2, 3, 7])
        elif where == "hdr":
            buf[o + rng.randint(5, 32)] ^= 1 << rng.randint(0, 7)
        elif where == "payload":
            buf[rng.randint(o + 33, e - 1)] ^= 1 << rng.randint(0, 7)
        elif where == "trailer":
            buf[e - rng.randint(1, 31)] ^= 0xFF
        else:
            buf[o + 21] ^= 1
    g = gpu_decode(gpu, buf, off)
    parsed, item_start, status = pyoracle.decode_blocks(buf, off)
    assert (status[1::2] == 0).all() and (status[0::2] != 0).all()
    compare_decode(g, parsed, item_start, status)


def test_structurally_broken_payloads_with_valid_checksums(gpu):
    """Payload corruption re-sealed with a correct header: exercises the parse
    validation (the reference would panic, lib.rs:62-66; both report PARSE)."""
    items = random_sorted_items(1200, seed=6)
    rng = random.Random(5)
    blocks = []
    for b in range(60):
        payload = bytearray(pyoracle.data_block_encode(items, b * 20, 20, restart_interval=rng.choice([1, 3, 16])))
        kind = b % 6
        if kind == 1:
            payload[rng.randrange(0, len(payload) - 31)] = rng.getrandbits(8)
        elif kind == 2:
            payload[-31] = 0  # restart interval 0
        elif kind == 3:
            payload[-4] ^= 1  # item count
        elif kind == 4:
            payload[-31 + 6] ^= 1  # binary index offset
        elif kind == 5:
            payload = payload[:rng.randint(0, 40)]
        blocks.append(pyoracle.block_write(bytes(payload)))
    buf, off = pack(blocks)
    for tuning in (None, (1, 256, 64), (48, 65536, 1024)):
        g = gpu_decode(gpu, buf, off, tuning=tuning)
        parsed, item_start, status = pyoracle.decode_blocks(buf, off)
        compare_decode(g, parsed, item_start, status)


def test_edge_handles(gpu):
    good = pyoracle.block_write(pyoracle.data_block_encode(pyoracle.Items.from_list([(b"k", b"v", 1, 0)])))
    blocks = [good, good[:10], b"", good[:33], pyoracle.block_write(b"x" * 40, 2), good]
    buf, off = pack(blocks)
    g = gpu_decode(gpu, buf, off)
    parsed, item_start, status = pyoracle.decode_blocks(buf, off)
    compare_decode(g, parsed, item_start, status)
    assert list(status) == [0, 8, 8, 4, 9, 0]
    # item capacity smaller than needed -> OVERFLOW on the clamped blocks
    g = gpu_decode(gpu, buf, off, item_cap=1)
    parsed, item_start, status = pyoracle.decode_blocks(buf, off, item_cap=1)
    compare_decode(g, parsed, item_start, status)


def test_round_trip_tombstones_and_big_seqnos(gpu):
    items = random_sorted_items(4000, seed=12, big_seq=True, vtypes=(0, 1, 2, 4))
    starts = pyoracle.cut_blocks(items, 1024)
    for ri, ratio in ((16, 0.0), (3, 2.5)):
        ref_buf, ref_off = pyoracle.encode_blocks(items, starts, restart_interval=ri, hash_ratio=ratio)
        buf, off, st = _gpu_encode(gpu, items, starts, ri, ratio, 0)
        assert (st == 0).all() and buf.tobytes() == ref_buf.tobytes()
        g = gpu_decode(gpu, buf, off)
        parsed, item_start, status = pyoracle.decode_blocks(buf, off)
        compare_decode(g, parsed, item_start, status)


def _mixed_items(n, seed):
    """Sorted items whose seqno varint length varies record to record (1-9
    bytes), keys 1-200 bytes (2-byte key lengths), values up to 300 bytes,
    all four value types: every header shape the decoder distinguishes."""
    rng = random.Random(seed)
    raw = {}
    while len(raw) < n:
        k = bytes(rng.choice(b"abcdefgh") for _ in range(rng.choice([rng.randint(1, 12), rng.randint(1, 200)])))
        s = rng.choice([rng.randint(0, 127), rng.randint(128, 1 << 14), rng.randint(1 << 14, 1 << 28),
                        rng.getrandbits(63)])
        t = rng.choice((0, 0, 0, 1, 2, 4))
        v = b"" if t in (1, 2) else bytes(rng.getrandbits(8) for _ in range(rng.choice([rng.randint(0, 20),
                                                                                         rng.randint(0, 300)])))
        raw[(k, s)] = (v, t)
    keys = sorted(raw, key=lambda ks: (ks[0], -ks[1]))
    return pyoracle.Items.from_list([(k, raw[(k, s)][0], s, raw[(k, s)][1]) for k, s in keys])


def _fuzz_blocks():
    """Valid payloads, then one structural mutation each (record bytes,
    varint continuation bits, binary-index entries incl. the first, item
    count, trailer marker), re-sealed with a correct checksum."""
    items = _mixed_items(6000, seed=21)
    rng = random.Random(77)
    blocks = []
    first = 0
    while first < items.n:
        cnt = min(rng.randint(1, 40), items.n - first)
        ri = rng.choice([1, 2, 4, 16, 32])
        payload = bytearray(pyoracle.data_block_encode(items, first, cnt, restart_interval=ri,
                                                       hash_ratio=rng.choice([0.0, 1.0])))
        first += cnt
        bin_len = int.from_bytes(payload[-29:-25], "little")
        bin_off = int.from_bytes(payload[-25:-21], "little")
        step = payload[-30]
        rec_end = bin_off - 1
        kind = rng.randrange(8)
        if kind == 1 and rec_end > 0:
            payload[rng.randrange(rec_end)] = rng.getrandbits(8)
        elif kind == 2 and rec_end > 0:
            payload[rng.randrange(rec_end)] |= 0x80
        elif kind == 3:
            r = rng.randrange(bin_len)
            v = int.from_bytes(payload[bin_off + r * step:bin_off + (r + 1) * step], "little")
            v = max(0, v + rng.choice([-2, -1, 1, 2]))
            payload[bin_off + r * step:bin_off + (r + 1) * step] = (v & ((1 << (8 * step)) - 1)).to_bytes(step, "little")
        elif kind == 4:
            payload[-4] = (payload[-4] + rng.choice([1, 255])) & 0xFF
        elif kind == 5:
            payload[rec_end] = rng.getrandbits(8)
        elif kind == 6 and rec_end > 1:
            for _ in range(2):
                payload[rng.randrange(rec_end)] ^= 1 << rng.randrange(8)
        blocks.append(pyoracle.block_write(bytes(payload)))
    return pack(blocks)


def test_resealed_mutation_fuzz(gpu):
    """The parser itself must reject or accept exactly as the oracle does."""
    buf, off = _fuzz_blocks()
    blocks = off[1:]
    parsed, item_start, status = pyoracle.decode_blocks(buf, off)
    assert (status == 0).sum() > len(blocks) // 4 and (status == 5).sum() > len(blocks) // 10
    for tuning in (None, (1, 256, 64), (8, 8192, 256), (48, 65536, 1024)):
        g = gpu_decode(gpu, buf, off, tuning=tuning)
        compare_decode(g, parsed, item_start, status)
