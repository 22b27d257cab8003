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
