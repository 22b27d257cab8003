"""CPU tests: the LZ4 block decoder oracle (oracle/lz4.c, test infrastructure)
pinned against liblz4 (pyarrow "lz4_raw", an independent implementation of the
block format lz4_flex decodes, src/table/block/mod.rs:104-118) and against the
branches of the format (tests/lz4_cases.py)."""
import numpy as np
import pytest

import pyoracle as o
from lz4_cases import handmade, lz4_compress

pa = pytest.importorskip("pyarrow")


@pytest.mark.parametrize("kind", ["zeros", "text", "random", "blocks"])
def test_oracle_matches_liblz4(kind):
    rng = np.random.default_rng(0)
    for n in (1, 15, 16, 100, 4096, 70000):
        if kind == "zeros":
            d = bytes(n)
        elif kind == "text":
            d = (b"the quick brown fox jumps over the lazy dog " * (n // 40 + 1))[:n]
        elif kind == "random":
            d = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        else:
            d = (bytes(range(16)) + rng.integers(0, 4, 48, dtype=np.uint8).tobytes()) * (n // 64 + 1)
            d = d[:n]
        c = lz4_compress(d)
        assert o.lz4_decompress(c, n) == d
        assert pa.Codec("lz4_raw").decompress(c, decompressed_size=n, asbytes=True) == d


@pytest.mark.parametrize("name,stream,exp", handmade(), ids=[c[0] for c in handmade()])
def test_oracle_handmade(name, stream, exp):
    # expected bytes by construction; liblz4 is not asked here because it also
    # enforces LZ4's end-of-block restrictions (last 5 bytes literals), which
    # these streams break on purpose and lz4_flex's decoder does not check
    assert o.lz4_decompress(stream, 1 << 16) == exp


def test_oracle_output_cap():
    d = b"abcdefgh" * 100
    c = lz4_compress(d)
    assert o.lz4_decompress(c, len(d)) == d
    assert o.lz4_decompress(c, len(d) - 1) is None  # would overrun uncompressed_length
