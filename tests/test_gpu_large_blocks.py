"""Data blocks above the general path's 72 KiB stage, up to the writer's 4 MiB
data-block target (use_data_block_size, src/table/writer/mod.rs:193-198):
encoded on the device bit-exact against the oracle two ways (pool=True: the
whole-GPU E3, record / tail / hash units and eight chains per block;
pool=False: one workgroup per block) and decoded two ways: with the workspace pool (pool=True, the default:
lsm_decode_workspace_size_ex) the blocks are cut into parse units (restart
intervals) and hash units (KiB blocks) over the whole GPU plus eight
single-wave XXH3 chains per block; without it (pool=False) each goes through
the stage in 64 KiB chunks on one workgroup (decode_chunked).
Cases: 256 KiB, 1 MiB and 4 MiB blocks, hash ratio 0 and 1.33 (the hash index
is dropped above 254 restart heads, trailer.rs:100-111), restart intervals 16
and 1, tombstones, a flipped payload bit (CKSUM) and a broken record re-sealed
with valid checksums (PARSE).  Bar: bit-exact bytes, statuses and fields."""
import numpy as np
import pytest

import pyoracle
from helpers import compare_decode, counter_items, gpu_decode, pack

pytestmark = pytest.mark.gpu


def _gpu_encode(gpu, items, starts, ri, ratio, pool=True):
    import torch
    d_items = gpu.items_to_device(items)
    d_starts = torch.from_numpy(np.asarray(starts, np.int64).astype(np.int32)).cuda()
    out = gpu.Encoder().encode(d_items, d_starts, len(starts) - 1, restart_interval=ri, hash_ratio=ratio, pool=pool)
    torch.cuda.synchronize()
    off = out["block_off"].cpu().numpy().view(np.uint64)
    return out["buf"].cpu().numpy()[:int(off[-1])], off, out["status"].cpu().numpy()[:len(starts) - 1]


@pytest.mark.parametrize("pool", [True, False])
@pytest.mark.parametrize("ratio", [0.0, 1.33])
@pytest.mark.parametrize("ri", [16, 1])
def test_large_data_blocks_round_trip(gpu, ri, ratio, pool):
    items = counter_items(80000, seed=41 + ri, tomb_frac=0.05)
    starts = np.array([0, 3300, 16400, 78200, 80000], np.uint32)  # ~256 KiB, 1 MiB, 4 MiB, ~130 KiB blocks
    ref_buf, ref_off = pyoracle.encode_blocks(items, starts, restart_interval=ri, hash_ratio=ratio)
    sizes = np.diff(ref_off.astype(np.int64))
    assert sizes.max() > 4_100_000 and (sizes > 72 * 1024).all(), sizes
    buf, off, st = _gpu_encode(gpu, items, starts, ri, ratio, pool)
    assert (st == 0).all() and (off == ref_off).all() and buf.tobytes() == ref_buf.tobytes()
    g = gpu_decode(gpu, buf, off, pool=pool)
    parsed, item_start, status = pyoracle.decode_blocks(buf, off)
    assert (status == 0).all()
    compare_decode(g, parsed, item_start, status)


@pytest.mark.parametrize("pool", [True, False])
def test_large_data_blocks_corrupted(gpu, pool):
    items = counter_items(20000, seed=7)
    starts = np.array([0, 16400, 20000], np.uint32)  # a 1 MiB and a ~300 KiB block
    buf, off = pyoracle.encode_blocks(items, starts)
    blocks = [bytes(buf[int(off[i]):int(off[i + 1])]) for i in range(2)]
    bad_ck = bytearray(blocks[0])
    bad_ck[33 + 700000] ^= 0x04  # a payload byte deep in the block: checksum mismatch
    rec = bytearray(blocks[0][33:])
    step, bin_off = rec[-30], int.from_bytes(rec[-25:-21], "little")  # trailer.rs:118-163
    start = int.from_bytes(rec[bin_off + step * 600:bin_off + step * 601], "little")
    rec[start] = 9  # restart head 600's value type: invalid
    late = bytearray(blocks[1][33:])
    late[-4] += 1  # item_count + 1: the last interval walks one record too many
    tests = blocks + [bytes(bad_ck), pyoracle.block_write(bytes(rec), 0), pyoracle.block_write(bytes(late), 0)]
    buf2, off2 = pack(tests)
    g = gpu_decode(gpu, buf2, off2, pool=pool)
    parsed, item_start, status = pyoracle.decode_blocks(buf2, off2)
    assert (status[:2] == 0).all() and status[2] == 4 and (status[3:] != 0).all(), status
    compare_decode(g, parsed, item_start, status)


@pytest.mark.parametrize("pool", [True, False])
@pytest.mark.parametrize("ratio", [0.0, 1.33])
def test_large_blocks_few_items(gpu, ratio, pool):
    """Blocks beyond the 96 KiB list image with at most 256 items (long values):
    E3 takes their record offsets from its own workgroup scan (E1 keeps full
    32-bit offsets only for blocks of more than 256 items); long seqnos and
    value lengths give multi-byte varints."""
    items = counter_items(400, key_len=24, val_len=3000, seqno=(1 << 40) + 5, seed=11, tomb_frac=0.1)
    starts = np.array([0, 40, 290, 400], np.uint32)  # ~110 KiB, ~680 KiB (250 items), ~300 KiB
    ref_buf, ref_off = pyoracle.encode_blocks(items, starts, restart_interval=16, hash_ratio=ratio)
    sizes = np.diff(ref_off.astype(np.int64))
    assert (sizes > 96 * 1024).all(), sizes
    buf, off, st = _gpu_encode(gpu, items, starts, 16, ratio, pool)
    assert (st == 0).all() and (off == ref_off).all() and buf.tobytes() == ref_buf.tobytes()
    g = gpu_decode(gpu, buf, off, pool=pool)
    parsed, item_start, status = pyoracle.decode_blocks(buf, off)
    assert (status == 0).all()
    compare_decode(g, parsed, item_start, status)


@pytest.mark.parametrize("pool", [True, False])
def test_huge_blocks_bad_binary_index(gpu, pool):
    """Re-sealed 1 MiB blocks whose binary index lies: two entries swapped (not
    monotone: the work kernel searches the index instead of the unit table),
    an entry moved to the next restart head's record, the last entry past the
    records, an entry 40 KiB late (past its next entries).  Statuses and fields
    match the oracle's."""
    items = counter_items(20000, seed=9)
    starts = np.array([0, 16400, 20000], np.uint32)
    buf, off = pyoracle.encode_blocks(items, starts)
    blocks = [bytes(buf[int(off[i]):int(off[i + 1])]) for i in range(2)]
    rec = bytes(blocks[0][33:])
    step, nint = rec[-30], int.from_bytes(rec[-29:-25], "little")  # trailer.rs:118-163
    bin_off = int.from_bytes(rec[-25:-21], "little")

    def ent(r, k):
        return int.from_bytes(r[bin_off + step * k:bin_off + step * (k + 1)], "little")

    def put(r, k, v):
        r[bin_off + step * k:bin_off + step * (k + 1)] = v.to_bytes(step, "little")

    cases = []
    r = bytearray(rec); a, b = ent(r, 300), ent(r, 301); put(r, 300, b); put(r, 301, a); cases.append(r)
    r = bytearray(rec); put(r, 500, ent(r, 501)); cases.append(r)
    r = bytearray(rec); put(r, nint - 1, bin_off + 8); cases.append(r)
    r = bytearray(rec); put(r, 640, ent(r, 640) + 40 * 1024); cases.append(r)
    tests = blocks + [pyoracle.block_write(bytes(c), 0) for c in cases]
    buf2, off2 = pack(tests)
    g = gpu_decode(gpu, buf2, off2, pool=pool)
    parsed, item_start, status = pyoracle.decode_blocks(buf2, off2)
    assert (status[:2] == 0).all() and (status[2:] != 0).all(), status
    compare_decode(g, parsed, item_start, status)


@pytest.mark.parametrize("pool", [True, False])
def test_huge_blocks_long_chains(gpu, pool):
    """A batch of ~3.7 MiB blocks (4096-step XXH3 chains) with a flipped payload
    bit (CKSUM) deep in a block, a broken record re-sealed (PARSE) and a trailer
    whose item count is one too many: statuses and fields as the oracle's."""
    items = counter_items(3 * 52429, seed=13)
    starts = np.array([0, 52429, 2 * 52429, 3 * 52429], np.uint32)
    buf, off = pyoracle.encode_blocks(items, starts)
    blocks = [bytes(buf[int(off[i]):int(off[i + 1])]) for i in range(3)]
    assert min(len(b) for b in blocks) > 3_500_000
    bad_ck = bytearray(blocks[0]); bad_ck[33 + 3_000_000] ^= 0x10
    rec = bytearray(blocks[1][33:])
    step, bin_off = rec[-30], int.from_bytes(rec[-25:-21], "little")
    st = int.from_bytes(rec[bin_off + step * 2000:bin_off + step * 2001], "little")
    rec[st] = 9  # a restart head's value type
    late = bytearray(blocks[2][33:]); late[-4] += 1
    tests = [blocks[0], bytes(bad_ck), pyoracle.block_write(bytes(rec), 0), pyoracle.block_write(bytes(late), 0),
             blocks[2]]
    buf2, off2 = pack(tests)
    g = gpu_decode(gpu, buf2, off2, pool=pool)
    parsed, item_start, status = pyoracle.decode_blocks(buf2, off2)
    assert status[0] == 0 and status[1] == 4 and (status[2:4] != 0).all() and status[4] == 0, status
    compare_decode(g, parsed, item_start, status)


def test_streamed_chains_pool_reuse(gpu):
    """Batches holding blocks of >= 2 MiB stream their XXH3 chains behind the
    parse units (unit-done flags in the pool).  One Decoder, so one pool, reused
    across calls with different blocks, statuses and expected types: a flag left
    by an earlier call must never pass for this call's (blocks whose trailer
    fails, or whose type differs, are hashed but not parsed)."""
    import torch
    items = counter_items(2 * 52429 + 3300, seed=17, tomb_frac=0.02)
    starts = np.array([0, 52429, 55729, 2 * 52429 + 3300], np.uint32)  # ~3.7 MiB, ~230 KiB, ~3.5 MiB
    buf, off = pyoracle.encode_blocks(items, starts)
    blocks = [bytes(buf[int(off[i]):int(off[i + 1])]) for i in range(3)]
    assert len(blocks[0]) > 2 * 1024 * 1024 and len(blocks[2]) > 2 * 1024 * 1024
    bad_ck = bytearray(blocks[2]); bad_ck[33 + 1_000_000] ^= 0x04
    late = bytearray(blocks[0][33:]); late[-4] += 1
    batches = [pack(blocks), pack([blocks[0], blocks[1], bytes(bad_ck)]),
               pack([pyoracle.block_write(bytes(late), 0), blocks[1], blocks[2]]), pack(blocks)]
    dec = gpu.Decoder()
    for buf2, off2 in batches:
        for et in (-1, 1, -1):
            n = len(off2) - 1
            d_blocks = gpu.to_device_bytes(buf2)
            d_off = torch.from_numpy(off2.astype(np.int64)).cuda()
            cap = len(buf2) // 3 + 1
            out = dec.alloc_outputs(cap, n)
            res = dec.decode(d_blocks, d_off, n, out, cap, et, pool=True)
            torch.cuda.synchronize()
            g = {k: v.cpu().numpy() for k, v in res.items()}
            g["status"] = g["status"][:n]
            parsed, item_start, status = pyoracle.decode_blocks(buf2, off2, expect_type=et)
            compare_decode(g, parsed, item_start, status)


def _mixed_batch(seed=5):
    """48 blocks of 80-400 KiB between 4 KiB blocks, and corrupted copies of
    some: header checksum (HDR_CKSUM), payload bit (CKSUM), broken record
    re-sealed (PARSE), item count + 1 re-sealed (trailer / PARSE), data_length
    (TRUNCATED), expected type (index block)."""
    r = np.random.default_rng(seed)
    cuts = [0]
    for i in range(48):
        cuts.append(cuts[-1] + 40)                          # ~4 KiB
        cuts.append(cuts[-1] + int(r.integers(900, 4600)))  # ~80-400 KiB
    items = counter_items(cuts[-1], seed=seed, tomb_frac=0.03)
    starts = np.array(cuts, np.uint32)
    buf, off = pyoracle.encode_blocks(items, starts)
    blocks = [bytes(buf[int(off[i]):int(off[i + 1])]) for i in range(len(starts) - 1)]
    big = [i for i, b in enumerate(blocks) if len(b) > 72 * 1024]
    assert len(big) >= 40
    out = list(blocks)
    b0 = bytearray(blocks[big[0]]); b0[10] ^= 0x01                 # header checksum
    b1 = bytearray(blocks[big[1]]); b1[33 + len(b1) // 2] ^= 0x20   # payload: CKSUM
    rec = bytearray(blocks[big[2]][33:])
    step, bin_off = rec[-30], int.from_bytes(rec[-25:-21], "little")
    st = int.from_bytes(rec[bin_off + step * 20:bin_off + step * 21], "little")
    rec[st] = 9                                                      # a restart head's value type
    late = bytearray(blocks[big[3]][33:]); late[-4] += 1             # item count + 1
    out += [bytes(b0), bytes(b1), pyoracle.block_write(bytes(rec), 0), pyoracle.block_write(bytes(late), 0),
            pyoracle.block_write(bytes(blocks[big[4]][33:]), 1)]       # type 1 with data records
    trunc = bytearray(blocks[big[5]]); trunc[21] ^= 0x01             # data_length field (header checksum too)
    out.append(bytes(trunc))
    return pack(out)


@pytest.mark.parametrize("pool", [True, False])
def test_huge_blocks_mixed_batch(gpu, pool):
    buf, off = _mixed_batch()
    g = gpu_decode(gpu, buf, off, pool=pool)
    parsed, item_start, status = pyoracle.decode_blocks(buf, off)
    assert (status[:-6] == 0).all() and (status[-6:] != 0).all(), status[-6:]
    compare_decode(g, parsed, item_start, status)
    for et in (0, 1):  # expected type: TYPE_MISMATCH wherever the type differs
        g = gpu_decode(gpu, buf, off, expect_type=et, pool=pool)
        parsed, item_start, status = pyoracle.decode_blocks(buf, off, expect_type=et)
        compare_decode(g, parsed, item_start, status)


@pytest.mark.parametrize("pool", [True, False])
@pytest.mark.parametrize("ratio", [0.0, 1.33])
def test_e1p_batch_with_small_blocks(gpu, ratio, pool):
    """A batch planned item-parallel (E1p: >= 4 Ki items per block on average)
    that also holds blocks of 1..300 items (the group kernel's packed record
    words, hash indexes) and blocks crossing many 64-item waves at odd
    offsets: bytes and offsets bit-exact against the oracle."""
    sizes = [50, 200, 20000, 7, 1, 30000, 300, 13, 9000, 64, 65, 129]
    items = counter_items(int(sum(sizes)), seed=21, tomb_frac=0.05)
    starts = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint32)
    assert sum(sizes) / len(sizes) >= 4096
    ref_buf, ref_off = pyoracle.encode_blocks(items, starts, restart_interval=16, hash_ratio=ratio)
    buf, off, st = _gpu_encode(gpu, items, starts, 16, ratio, pool)
    assert (st == 0).all() and (off == ref_off).all() and buf.tobytes() == ref_buf.tobytes()


def test_huge_blocks_pool_sizes(gpu):
    """A pool too small for every huge block of the batch: the blocks whose
    contributions do not fit take the one-workgroup path; results unchanged."""
    buf, off = _mixed_batch(seed=9)
    parsed, item_start, status = pyoracle.decode_blocks(buf, off)
    n = len(off) - 1
    base = gpu.lib().lsm_decode_workspace_size(n)
    full = gpu.lib().lsm_decode_workspace_size_ex(n, len(buf) + 64)
    assert full > base
    for extra in (0, 100, 4096, 40000, 300_000, 1_500_000, full - base):
        g = gpu_decode(gpu, buf, off, workspace_bytes=base + extra)
        compare_decode(g, parsed, item_start, status)


def test_huge_blocks_payload_verified(gpu):
    """LSM_DECODE_PAYLOAD_VERIFIED (frames whose checksum the LZ4 path already
    checked): no payload hash; trailer / parse statuses as the oracle's."""
    buf, off = _mixed_batch(seed=13)
    parsed, item_start, status = pyoracle.decode_blocks(buf, off)
    keep = [i for i in range(len(off) - 1) if status[i] != 4]  # drop the CKSUM block
    blocks = [bytes(buf[int(off[i]):int(off[i + 1])]) for i in keep]
    buf2, off2 = pack(blocks)
    parsed, item_start, status = pyoracle.decode_blocks(buf2, off2)
    for pool in (True, False):
        g = gpu_decode(gpu, buf2, off2, tuning=(0, 0, 0, gpu.DECODE_PAYLOAD_VERIFIED), pool=pool)
        compare_decode(g, parsed, item_start, status)


@pytest.mark.parametrize("pool", [True, False])
def test_huge_blocks_encode_mixed(gpu, pool):
    """~48 blocks of 80-400 KiB between 4 KiB blocks (hash ratio 1.33: the small
    blocks carry a hash index, the huge ones drop it): bytes == oracle."""
    r = np.random.default_rng(3)
    cuts = [0]
    for i in range(48):
        cuts.append(cuts[-1] + 40)
        cuts.append(cuts[-1] + int(r.integers(900, 4600)))
    items = counter_items(cuts[-1], seed=3, tomb_frac=0.03)
    starts = np.array(cuts, np.uint32)
    ref_buf, ref_off = pyoracle.encode_blocks(items, starts, restart_interval=16, hash_ratio=1.33)
    buf, off, st = _gpu_encode(gpu, items, starts, 16, 1.33, pool)
    assert (st == 0).all() and (off == ref_off).all() and buf.tobytes() == ref_buf.tobytes()


@pytest.mark.parametrize("pool", [True, False])
def test_huge_index_blocks_encode(gpu, pool):
    """Full block indexes over 96 KiB (restart interval 1, u64 handles)."""
    import torch
    from helpers import index_items
    items = index_items(14000, seed=11)
    starts = np.array([0, 6000, 6001, 14000], np.uint32)
    ref_buf, ref_off = pyoracle.encode_blocks(items, starts, block_type=1)
    d_items = gpu.items_to_device(items)
    d_starts = torch.from_numpy(starts.astype(np.int32)).cuda()
    out = gpu.Encoder().encode(d_items, d_starts, 3, restart_interval=1, block_type=1, pool=pool)
    torch.cuda.synchronize()
    off = out["block_off"].cpu().numpy().view(np.uint64)
    assert (out["status"].cpu().numpy()[:3] == 0).all() and (off == ref_off).all()
    assert out["buf"].cpu().numpy()[:int(off[-1])].tobytes() == ref_buf.tobytes()


def test_huge_encode_pool_sizes(gpu):
    """Encode with a pool too small for every huge block of the batch: the blocks
    past the pool's capacity are written by the one-workgroup E3; bytes unchanged."""
    import torch
    items = counter_items(80000, seed=19)
    starts = np.array([0, 3300, 16400, 30000, 47000, 78200, 80000], np.uint32)
    ref_buf, ref_off = pyoracle.encode_blocks(items, starts)
    d_items = gpu.items_to_device(items)
    d_starts = torch.from_numpy(starts.astype(np.int32)).cuda()
    nb = len(starts) - 1
    n = items.n
    import ctypes
    bound = gpu.lib().lsm_encode_bound(n, nb, int(d_items["keys"].numel()), int(d_items["vals"].numel()),
                                       ctypes.byref(gpu.LsmBlockParams(16, gpu.BLOCK_DATA, 0, 0, 0.0)))
    base = gpu.lib().lsm_encode_workspace_size(n, nb)
    full = gpu.lib().lsm_encode_workspace_size_ex(n, nb, bound)
    for extra in (0, 5000, 60000, 300_000, 1_500_000, full - base):
        out = gpu.Encoder().encode(d_items, d_starts, nb, workspace_bytes=base + extra, pool=True)
        torch.cuda.synchronize()
        off = out["block_off"].cpu().numpy().view(np.uint64)
        assert (out["status"].cpu().numpy()[:nb] == 0).all() and (off == ref_off).all(), extra
        assert out["buf"].cpu().numpy()[:int(off[-1])].tobytes() == ref_buf.tobytes(), extra


def test_huge_encode_concurrent_streams(gpu):
    """Two host threads encoding ragged pool batches (group-class, listed and
    huge blocks) on two streams at once, each through its own Encoder, five
    times: bytes, offsets and statuses == the oracle's."""
    import threading
    import torch
    sizes = [50, 200, 20000, 7, 1, 30000, 300, 13, 9000, 64, 65, 129, 2500, 16400]
    cases = []
    for seed in (31, 32):
        items = counter_items(int(sum(sizes)), seed=seed, tomb_frac=0.05)
        starts = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint32)
        ref_buf, ref_off = pyoracle.encode_blocks(items, starts)
        d_items = gpu.items_to_device(items)
        d_starts = torch.from_numpy(starts.astype(np.int32)).cuda()
        cases.append((d_items, d_starts, len(starts) - 1, ref_buf, ref_off))
    torch.cuda.synchronize()

    def check(out, nb, ref_buf, ref_off):
        off = out["block_off"].cpu().numpy().view(np.uint64)
        assert (out["status"].cpu().numpy()[:nb] == 0).all() and (off == ref_off).all()
        assert out["buf"].cpu().numpy()[:int(off[-1])].tobytes() == ref_buf.tobytes()

    results, errors = [None, None], []

    def worker(t):
        try:
            d_items, d_starts, nb, _, _ = cases[t]
            s = torch.cuda.Stream()
            enc = gpu.Encoder()
            with torch.cuda.stream(s):
                out = enc.encode(d_items, d_starts, nb, pool=True)
                for _ in range(4):
                    out["buf"].zero_()
                    enc.encode(d_items, d_starts, nb, out=out, stream=s, pool=True)
            s.synchronize()
            results[t] = out
        except Exception as e:  # (reported by the main thread)
            errors.append(e)

    threads = [threading.Thread(target=worker, args=(t,)) for t in range(2)]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    assert not errors, errors
    for t in range(2):
        check(results[t], cases[t][2], cases[t][3], cases[t][4])



# Diagnostic build (-DLSM_DIAG, lsm-tree_amd/.variants/libdiag.so, built by
# __graft_entry__.build()): decode flag bits that force the streamed chains'
# give-up path deterministically (csrc/decode.hpp).
DIAG_STREAM_GIVE_UP = 0x4000
DIAG_NO_CHAIN_FALLBACK = 0x8000


def test_streamed_chain_give_up(gpu, diag_lib):
    """The streamed huge-block chains give a block up after 5 ms without progress
    (other streams holding the CUs); the diagnostic flag makes every chain wave
    give up at its first wait.  With the call's fallback chain pass every status
    and row equals the oracle's (a give-up is never reported as a checksum
    mismatch, block/mod.rs:141-149); with the pass skipped, exactly the blocks
    whose chains gave up carry LSM_INCOMPLETE."""
    items = counter_items(2 * 52429 + 3300, seed=29, tomb_frac=0.02)
    starts = np.array([0, 52429, 55729, 2 * 52429 + 3300], np.uint32)  # ~3.7 MiB, ~230 KiB, ~3.5 MiB
    buf, off = pyoracle.encode_blocks(items, starts)
    blocks = [bytes(buf[int(off[i]):int(off[i + 1])]) for i in range(3)]
    bad_ck = bytearray(blocks[2]); bad_ck[33 + 1_500_000] ^= 0x08
    late = bytearray(blocks[0][33:]); late[-4] += 1
    buf2, off2 = pack([blocks[0], blocks[1], bytes(bad_ck), pyoracle.block_write(bytes(late), 0), blocks[2]])
    parsed, item_start, status = pyoracle.decode_blocks(buf2, off2)
    assert list(status[:3]) == [0, 0, 4] and status[3] != 0 and status[4] == 0, status
    saved = gpu._lib
    gpu._lib = diag_lib
    try:
        g = gpu_decode(gpu, buf2, off2, tuning=(0, 0, 0, DIAG_STREAM_GIVE_UP), pool=True)
        compare_decode(g, parsed, item_start, status)
        g2 = gpu_decode(gpu, buf2, off2, tuning=(0, 0, 0, DIAG_STREAM_GIVE_UP | DIAG_NO_CHAIN_FALLBACK), pool=True)
        g3 = gpu_decode(gpu, buf2, off2, pool=True)  # the diagnostic build without the flags: as the release
        compare_decode(g3, parsed, item_start, status)
    finally:
        gpu._lib = saved
    assert gpu.STATUS[13] == "INCOMPLETE"
    # every block here has a valid header, so every one is a streamed huge block
    assert (g2["status"] == 13).all(), g2["status"]
