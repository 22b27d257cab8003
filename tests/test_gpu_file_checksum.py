"""GPU whole-file checksum (lsm_xxh3_128_file) against the oracle's xxh3_128:
the ChecksummedWriter digest of an SST file (src/checksum.rs:59-96) equals the
one-shot xxh3_128 of the file (tests/table_full_file_checksum.rs:26-31).
Bar: bit-exact 128-bit digests, every XXH3 size class and start alignment."""
import random

import numpy as np
import pytest

import pyoracle

pytestmark = pytest.mark.gpu

SIZES = [0, 1, 3, 4, 8, 9, 16, 17, 128, 129, 240, 241, 1023, 1024, 1025, 1088, 2048, 4103, 65599,
         (256 << 10) + 1, (512 << 10) + 1, 1 << 20, (1 << 20) + 1, (3 << 20) + 333]


def test_file_checksum_sizes(gpu):
    import torch
    rng = np.random.default_rng(7)
    data = rng.integers(0, 256, (4 << 20) + 64, dtype=np.uint8)
    d = torch.from_numpy(data).cuda()
    r = random.Random(3)
    for n in SIZES:
        off = r.randrange(16)
        got = gpu.xxh3_128_file(d, n, off)
        exp = pyoracle.xxh3_128(data[off:off + n].tobytes())
        assert (got[1] << 64) | got[0] == exp, n


def test_file_checksum_sst_sized(gpu):
    """A 64 MiB "table" (the flush target, src/tree/mod.rs:374-377) of encoded blocks."""
    import torch
    rng = np.random.default_rng(11)
    n = (64 << 20) + 12345
    data = rng.integers(0, 256, n + 64, dtype=np.uint8)
    got = gpu.xxh3_128_file(torch.from_numpy(data).cuda(), n)
    assert (got[1] << 64) | got[0] == pyoracle.xxh3_128(data[:n].tobytes())


def _chunkings(total, r):
    """Split points for one file: single bytes, sizes < 240, runs straddling and
    ending on KiB boundaries, big pieces, empty writes."""
    yield [total]
    yield [1] * min(total, 300) + ([total - 300] if total > 300 else [])
    for _ in range(3):
        cuts, left = [], total
        while left:
            kind = r.randrange(6)
            n = (r.randrange(1, 240) if kind == 0 else r.choice([1023, 1024, 1025, 64, 63, 65]) if kind == 1
                 else r.randrange(1, 5000) if kind == 2 else r.randrange(1, 1 << 17) if kind == 3
                 else 0 if kind == 4 else 1024 - ((total - left) % 1024) or 1024)
            n = min(n, left)
            cuts.append(n)
            left -= n
        yield cuts


@pytest.mark.parametrize("total", [0, 1, 100, 240, 241, 1000, 1024, 1025, 2048, 2049, 5000, 65536 + 7, 300000])
def test_stream_checksum_random_chunkings(gpu, total):
    """ChecksummedWriter::write in pieces (src/checksum.rs:92-95) then checksum():
    equal to the oracle's one-shot xxh3_128 of the concatenation for every split,
    and digest() can be taken mid-stream (the running state is not consumed)."""
    import torch
    rng = np.random.default_rng(total + 5)
    data = rng.integers(0, 256, total + 64, dtype=np.uint8)
    d = torch.from_numpy(data).cuda()
    r = random.Random(total)
    for cuts in _chunkings(total, r):
        w = gpu.ChecksummedWriter()
        pos = 0
        for i, n in enumerate(cuts):
            w.write(d, n, pos)
            pos += n
            if i % 7 == 3:  # a digest in the middle of the stream
                got = w.checksum()
                assert (got[1] << 64) | got[0] == pyoracle.xxh3_128(data[:pos].tobytes()), (cuts[:i + 1], pos)
        assert pos == total
        got = w.checksum()
        assert (got[1] << 64) | got[0] == pyoracle.xxh3_128(data[:total].tobytes()), cuts


def test_stream_checksum_sst_writer_order(gpu, oracle):
    """The writer's own order: data blocks flushed one spill at a time, then the
    index, then a trailing region (writer/mod.rs:303-366, 371-539); the running
    checksum equals xxh3_128 of the assembled file."""
    import torch
    rng = np.random.default_rng(21)
    pieces = [rng.integers(0, 256, int(n), dtype=np.uint8) for n in rng.integers(3000, 70000, 40)]
    pieces += [rng.integers(0, 256, 12345, dtype=np.uint8), rng.integers(0, 256, 77, dtype=np.uint8)]
    w = gpu.ChecksummedWriter()
    for p in pieces:
        w.write(torch.from_numpy(np.concatenate([p, np.zeros(64, np.uint8)])).cuda(), len(p))
    got = w.checksum()
    whole = np.concatenate(pieces)
    assert (got[1] << 64) | got[0] == pyoracle.xxh3_128(whole.tobytes())
    assert w.bytes_written == len(whole)


def _batch_round(torch, files, pos, cuts, pad=64):
    """One update_batch round: state i gets files[i][pos[i] .. pos[i] + cuts[i])."""
    parts, off = [], [0]
    for f, p, c in zip(files, pos, cuts):
        parts.append(f[p:p + c])
        off.append(off[-1] + c)
    arena = np.concatenate(parts + [np.zeros(pad, np.uint8)])
    return torch.from_numpy(arena).cuda(), torch.tensor(off, dtype=torch.int64, device="cuda"), off[-1]


def test_stream_batch_random_chunkings(gpu):
    """64 running checksums advanced together (lsm_xxh3_128_stream_update_batch:
    the ChecksummedWriter of every table of a MultiWriter, multi_writer.rs:181-257):
    random per-state chunk sizes (empty, < 240 B, KiB-straddling, large) over 6
    rounds; mid-stream digests after round 3 and final digests equal the oracle's
    one-shot xxh3_128 of each file."""
    import torch
    rng = np.random.default_rng(99)
    r = random.Random(99)
    n = 64
    sizes = [r.choice([0, 1, 239, 240, 241, 1023, 1024, 1025, r.randrange(1, 5000), r.randrange(1, 400000)])
             for _ in range(n)]
    files = [rng.integers(0, 256, s, dtype=np.uint8) for s in sizes]
    ws = gpu.ChecksummedWriterSet(n)
    pos = [0] * n
    for rnd in range(6):
        cuts = []
        for i in range(n):
            left = sizes[i] - pos[i]
            c = left if rnd == 5 else min(left, r.choice([0, 1, 63, 1024, r.randrange(0, 3000), r.randrange(0, 1 << 17)]))
            cuts.append(c)
        d, off, total = _batch_round(torch, files, pos, cuts)
        st = ws.write(d, off, total).cpu().numpy()[:n]
        assert (st == 0).all(), st
        pos = [p + c for p, c in zip(pos, cuts)]
        if rnd == 2:
            got = ws.checksums()
            for i in range(n):
                assert (got[i][1] << 64) | got[i][0] == pyoracle.xxh3_128(files[i][:pos[i]].tobytes()), (i, pos[i])
    assert pos == sizes
    got = ws.checksums()
    for i in range(n):
        assert (got[i][1] << 64) | got[i][0] == pyoracle.xxh3_128(files[i].tobytes()), (i, sizes[i])


def test_stream_batch_bad_states(gpu):
    """A state never initialised and a decreasing range get LSM_BAD_ARG and stay
    unchanged; the other states advance; a total_len below the ranges' bytes
    rejects the whole call."""
    import torch
    rng = np.random.default_rng(5)
    files = [rng.integers(0, 256, 5000, dtype=np.uint8) for _ in range(4)]
    ws = gpu.ChecksummedWriterSet(4)
    size = gpu.lib().lsm_xxh3_128_stream_state_size()
    ws.states[size:2 * size].zero_()  # state 1: not initialised (no magic)
    arena = np.concatenate(files + [np.zeros(64, np.uint8)])
    d = torch.from_numpy(arena).cuda()
    off = torch.tensor([0, 5000, 10000, 15000, 14000], dtype=torch.int64, device="cuda")  # state 3: decreasing
    st = ws.write(d, off, 20000).cpu().numpy()
    assert list(st) == [0, 10, 0, 10]
    got = ws.checksums()
    for i in (0, 2):
        assert (got[i][1] << 64) | got[i][0] == pyoracle.xxh3_128(files[i].tobytes())
    assert (got[3][1] << 64) | got[3][0] == pyoracle.xxh3_128(b"")
    # ranges of 20000 bytes against total_len 1000: nothing changes
    off2 = torch.tensor([0, 5000, 10000, 15000, 20000], dtype=torch.int64, device="cuda")
    st = ws.write(d, off2, 1000).cpu().numpy()
    assert list(st) == [10, 10, 10, 10]
    got2 = ws.checksums()
    assert got2[0] == got[0] and got2[2] == got[2] and got2[3] == got[3]
    # ranges only a few bytes over total_len (within the workspace's KiB-block
    # slack): still the whole call is rejected, as lsmgpu.h states
    for total in (19997, 19999):
        st = ws.write(d, off2, total).cpu().numpy()
        assert list(st) == [10, 10, 10, 10], total
        assert ws.checksums() == got2
    # one state, total_len 0, a 2000-byte range (the advisor's example)
    one = gpu.ChecksummedWriterSet(1)
    off1 = torch.tensor([0, 2000], dtype=torch.int64, device="cuda")
    assert list(one.write(d, off1, 0).cpu().numpy()) == [10]
    assert (lambda c: (c[1] << 64) | c[0])(one.checksums()[0]) == pyoracle.xxh3_128(b"")
    # exactly total_len bytes: accepted
    st = ws.write(d, off2, 20000).cpu().numpy()
    assert list(st) == [0, 10, 0, 0]
