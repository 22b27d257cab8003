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
