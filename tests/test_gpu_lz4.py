"""GPU parity of batched LZ4 block decompression (lsm_lz4_decompress_blocks,
Block::from_reader with CompressionType::Lz4, src/table/block/mod.rs:87-128)
against the oracle (oracle/lz4.c).  Inputs: real data blocks (oracle-encoded)
compressed by liblz4, every size class the kernels split on (small LDS path,
large LDS path, serial HBM path), hand-built streams for every branch of the
format, and corrupted headers / checksums / streams.
Bar: bit-exact decompressed bytes and identical per-block status."""
import numpy as np
import pytest

import pyoracle
from helpers import counter_items, random_sorted_items
from lz4_cases import handmade, lz4_compress, seq

pytestmark = pytest.mark.gpu

OK, CKSUM, HDR_CKSUM, BAD_MAGIC, OVERFLOW, DECOMPRESS = 0, 4, 3, 1, 6, 12


def _frame(stored: bytes, raw_len: int, block_type=0) -> bytes:
    return pyoracle.block_header(block_type, stored, raw_len) + stored


def _run(gpu, blocks):
    """blocks: list of on-disk block bytes -> (list of decoded bytes, status list)."""
    import torch
    pad = list(blocks)
    off = np.zeros(len(pad) + 1, np.int64)
    off[1:] = np.cumsum([len(b) for b in pad])
    buf = gpu.to_device_bytes(np.frombuffer(b"".join(pad), np.uint8))
    out, out_off, status = gpu.lz4_decompress_blocks(buf, torch.from_numpy(off).cuda())
    torch.cuda.synchronize()
    o = out.cpu().numpy().tobytes()
    oo = out_off.cpu().numpy()
    return [o[oo[i]:oo[i + 1]] for i in range(len(blocks))], status.cpu().numpy().tolist()


def _payloads(n_items, restart, kind, seed):
    items = (random_sorted_items if kind == "random" else counter_items)(n_items, seed=seed)
    return pyoracle.data_block_encode(items, restart_interval=restart)


def test_lz4_real_blocks_all_size_classes(gpu):
    raws = []
    for n_items, kind in [(52, "counter"), (52, "random"), (205, "counter"), (820, "counter"),
                          (820, "random"), (1300, "counter")]:  # 4 KiB .. ~100 KiB payloads
        raws.append(_payloads(n_items, 16, kind, n_items))
    rng = np.random.default_rng(9)
    raws += [rng.integers(0, 256, 5000, dtype=np.uint8).tobytes(),  # incompressible
             bytes(9000), b"z"]
    blocks = [_frame(lz4_compress(r), len(r)) for r in raws]
    got, st = _run(gpu, blocks)
    assert st == [OK] * len(blocks)
    for g, r in zip(got, raws):
        assert g == r
        assert pyoracle.lz4_decompress(lz4_compress(r), len(r)) == r


def test_lz4_many_small_blocks(gpu):
    raws = [_payloads(52, ri, "random", s) for s, ri in enumerate([1, 2, 4, 8, 16] * 40)]
    blocks = [_frame(lz4_compress(r), len(r)) for r in raws]
    got, st = _run(gpu, blocks)
    assert st == [OK] * len(raws) and got == raws


def test_lz4_handmade_streams(gpu):
    cases = handmade()
    blocks, exp_bytes, exp_st = [], [], []
    for name, stream, exp in cases:
        raw_len = len(exp) if exp is not None else 64
        blocks.append(_frame(stream, raw_len))
        exp_bytes.append(exp)
        exp_st.append(OK if exp is not None else DECOMPRESS)
    # the same streams behind a 10 KiB literal run + one match, so the large-class
    # kernel (LDS stages > 8 KiB) decodes them too
    big = bytes(range(256)) * 40
    prefix, prefix_bytes = seq(big, 256, 4), big + big[len(big) - 256:len(big) - 252]
    for name, stream, exp in cases:
        if exp is None or not stream:
            continue
        blocks.append(_frame(prefix + stream, len(prefix_bytes) + len(exp)))
        exp_bytes.append(prefix_bytes + exp)
        exp_st.append(OK)
    got, st = _run(gpu, blocks)
    assert st == exp_st
    for g, e, s in zip(got, exp_bytes, st):
        if s == OK:
            assert g == e


def test_lz4_status_codes(gpu):
    r = _payloads(52, 16, "counter", 1)
    c = lz4_compress(r)
    good = _frame(c, len(r))
    bad_ck = bytearray(good)
    bad_ck[40] ^= 1  # payload byte: checksum mismatch
    bad_hdr = bytearray(good)
    bad_hdr[30] ^= 1  # header checksum
    bad_magic = bytearray(good)
    bad_magic[0] = ord("X")
    short = _frame(c, len(r) + 7)  # uncompressed_length larger than the stream decodes to
    got, st = _run(gpu, [good, bytes(bad_ck), bytes(bad_hdr), bytes(bad_magic), short])
    assert st == [OK, CKSUM, HDR_CKSUM, BAD_MAGIC, DECOMPRESS]
    assert got[0] == r


def test_lz4_corrupt_length_cannot_size_the_output(gpu):
    """A bit flip in uncompressed_length (header bytes 25-28) is a header-checksum
    failure, reported per block without the corrupt length sizing the output
    (Block::from_reader allocates only after Header::decode_from passed,
    block/mod.rs:91-112).  A verified length above the caller's cap is OVERFLOW;
    a handle shorter than a header is TRUNCATED."""
    r = _payloads(52, 16, "counter", 2)
    good = _frame(lz4_compress(r), len(r))
    huge = bytearray(good)
    huge[28] ^= 0x80  # uncompressed_length += 2 GiB, header checksum now stale
    got, st = _run(gpu, [good, bytes(huge), good])
    assert st == [OK, HDR_CKSUM, OK] and got[0] == r and got[2] == r and got[1] == b""
    # a correctly sealed header claiming 1 GiB: within the cap it is sized, above it OVERFLOW
    import torch
    big = _frame(lz4_compress(r), 1 << 30)
    buf = gpu.to_device_bytes(np.frombuffer(big + good, np.uint8))
    off = torch.tensor([0, len(big), len(big) + len(good)], dtype=torch.int64).cuda()
    out, out_off, status = gpu.lz4_decompress_blocks(buf, off, max_block_bytes=1 << 20)
    torch.cuda.synchronize()
    assert status.cpu().tolist() == [OVERFLOW, OK] and out_off.cpu().tolist() == [0, 0, len(r)]
    # truncated handles: fewer bytes than a header
    buf = gpu.to_device_bytes(np.frombuffer(good[:20] + good, np.uint8))
    off = torch.tensor([0, 20, 20 + len(good)], dtype=torch.int64).cuda()
    out, out_off, status = gpu.lz4_decompress_blocks(buf, off)
    torch.cuda.synchronize()
    assert status.cpu().tolist()[1] == OK and status.cpu().tolist()[0] != OK and int(out_off[1]) == 0


def test_lz4_chained_parse(gpu):
    """LZ4 -> parse chaining: Block::from_reader(Lz4) then DataBlock::new + iter
    (block/mod.rs:104-118, data_block/mod.rs:335,476) on the device:
    lsm_lz4_plan_framed -> lsm_lz4_decompress_framed -> lsm_decode_blocks_tuned with
    LSM_DECODE_PAYLOAD_VERIFIED.  Every parsed field must equal the oracle's decode of the
    uncompressed payload; corrupt stored bytes keep their checksum status, a malformed
    stream its DECOMPRESS status, a bad type its TYPE_MISMATCH."""
    import torch
    from helpers import FIELD_VIEW, prefix_items
    raws = []
    for n_items, kind, ri in [(52, "counter", 16), (52, "random", 1), (205, "counter", 16), (820, "counter", 16),
                              (820, "random", 4), (1300, "counter", 16)]:
        raws.append(_payloads(n_items, ri, kind, n_items))
    raws += [pyoracle.data_block_encode(prefix_items(56, seed=s)) for s in range(8)]
    raws += [_payloads(52, 16, "counter", 100 + s) for s in range(40)]
    blocks = [_frame(lz4_compress(r), len(r)) for r in raws]
    # corruptions: stored-byte flip (CKSUM), malformed stream (DECOMPRESS), index type (TYPE_MISMATCH)
    bad_ck = bytearray(blocks[3]); bad_ck[40] ^= 1; blocks[3] = bytes(bad_ck)
    blocks[7] = _frame(b"\xf0", len(raws[7]))
    blocks[9] = _frame(lz4_compress(raws[9]), len(raws[9]), block_type=1)
    off = np.zeros(len(blocks) + 1, np.int64)
    off[1:] = np.cumsum([len(b) for b in blocks])
    buf = gpu.to_device_bytes(np.frombuffer(b"".join(blocks), np.uint8))
    out = gpu.decode_lz4_blocks(buf, torch.from_numpy(off).cuda(), expect_type=0)
    torch.cuda.synchronize()
    st = out["status"].cpu().numpy()[:len(blocks)]
    want = [OK] * len(blocks)
    want[3], want[7], want[9] = CKSUM, DECOMPRESS, 7
    assert st.tolist() == want
    # without the status merge: a block whose decompression failed still reports an
    # error from the decode alone (its frame header is all zero: BAD_MAGIC), never OK
    dst = out["decode_status"].cpu().numpy()[:len(blocks)]
    assert dst[3] == BAD_MAGIC and dst[7] == BAD_MAGIC and dst[9] == 7
    fr = out["frames"].cpu().numpy()
    fo = out["frame_off"].cpu().numpy()
    assert not fr[fo[3]:fo[3] + 33].any() and not fr[fo[7]:fo[7] + 33].any()
    starts = out["item_start"].cpu().numpy().view(np.uint32)
    frames = out["frames"].cpu().numpy()
    foff = out["frame_off"].cpu().numpy()
    for b, r in enumerate(raws):
        if want[b] != OK:
            continue
        assert frames[foff[b] + 33:foff[b + 1]].tobytes() == r
        n, parsed = pyoracle.data_block_decode(r)
        lo, hi = int(starts[b]), int(starts[b + 1])
        assert hi - lo == n
        for f, dt in FIELD_VIEW.items():
            if f != "handle_off":
                assert (out[f].cpu().numpy().view(dt)[lo:hi] == parsed[f].astype(dt)).all(), (b, f)
    # the frame header is a well-formed uncompressed-size header of the stored checksum
    st0, h = pyoracle.header_decode(frames[foff[0]:foff[0] + 33].tobytes())
    assert st0 == 0 and h.data_length == len(raws[0]) == h.uncompressed_length


def test_lz4_chain_capped_no_sync(gpu):
    """lsm_lz4_plan_capped (framed): a frame arena sized without reading the plan
    back.  Exactly large enough: the same statuses and fields as the synchronising
    chain; one byte short: every block reports OVERFLOW and no frame is written."""
    import torch
    raws = [_payloads(52, 16, "counter", 200 + s) for s in range(20)] + [_payloads(820, 4, "random", 7)]
    blocks = [_frame(lz4_compress(r), len(r)) for r in raws]
    off = np.zeros(len(blocks) + 1, np.int64)
    off[1:] = np.cumsum([len(b) for b in blocks])
    buf = gpu.to_device_bytes(np.frombuffer(b"".join(blocks), np.uint8))
    d_off = torch.from_numpy(off).cuda()
    ref = gpu.decode_lz4_blocks(buf, d_off, expect_type=0)
    torch.cuda.synchronize()
    total = int(ref["frame_off"][-1].item())
    n_items = int(ref["item_start"][len(blocks)].item())
    got = gpu.decode_lz4_blocks(buf, d_off, expect_type=0, frames_cap=total)
    torch.cuda.synchronize()
    assert (got["status"][:len(blocks)] == 0).all() and (ref["status"][:len(blocks)] == 0).all()
    assert torch.equal(got["frame_off"], ref["frame_off"])
    for f in ("seqno", "key_off", "val_off", "val_len", "key_len", "prefix_len", "vtype"):
        assert torch.equal(got[f][:n_items], ref[f][:n_items]), f
    short = gpu.decode_lz4_blocks(buf, d_off, expect_type=0, frames_cap=total - 1)
    torch.cuda.synchronize()
    assert (short["status"][:len(blocks)] == 6).all()  # LSM_OVERFLOW
    assert (short["frame_off"] == 0).all() and int((short["frames"] != 0).sum().item()) == 0
