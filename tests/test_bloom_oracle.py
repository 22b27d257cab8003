"""CPU tests: pin the Bloom-filter oracle (oracle/bloom.c, test infrastructure)
to the reference's own known answers and properties.

Reference tests mirrored (fjall-rs/lsm-tree 3.1.9):
  src/table/filter/standard_bloom/builder.rs:173-187  calculate_m KATs
  src/table/filter/bit_array/builder.rs:48-71         bit order (MSB first)
  src/table/filter/standard_bloom/mod.rs:127-305      round trip, members, FPR bands
  src/table/filter/mod.rs:92-115                      estimated sizes (m per policy)
"""
import random
import string

import numpy as np
import pytest

import pyoracle as o


def _h(keys):
    return np.array([o.xxh3_64(k) for k in keys], np.uint64)


def _nanoids(n, seed):
    r = random.Random(seed)
    alpha = string.ascii_letters + string.digits + "_-"  # nanoid's default alphabet, 21 chars
    return [''.join(r.choice(alpha) for _ in range(21)).encode() for _ in range(n)]


def test_calculate_m_kats():
    assert o.bloom_calculate_m(1_000, 0.01) == 9_592
    assert o.bloom_calculate_m(1_000, 0.1) == 4_800
    assert o.bloom_calculate_m(1_000_000, 0.1) == 4_792_536


def test_policy_shapes():
    # BitsPerKey(10.0) over 1M keys: 1.25 MB of bits (filter/mod.rs:92-101), k = (10 ln2) as usize
    m, k = o.bloom_shape(1_000_000, bpk=10.0)
    assert (m // 8, k) == (1_250_000, 6)
    m, k = o.bloom_shape(1_000_000, fpr=0.01)
    assert 1_100_000 < m // 8 < 1_300_000
    m, k = o.bloom_shape(3, bpk=5.0)  # bytes = ceil(15/8) = 2 -> m = 16
    assert (m, k) == (16, 3)
    with pytest.raises(ValueError):
        o.bloom_shape(0, bpk=10.0)


def test_bit_order_msb_first():
    # bit_array/builder.rs:48-71: bit 0 is 0x80 of byte 0, bit 7 is 0x01.  A
    # filter with k=1, m=16 and hash h sets exactly bit h % 16.
    for h, byte, mask in [(0, 0, 0x80), (7, 0, 0x01), (1, 0, 0x40), (9, 1, 0x40), (16 + 6, 0, 0x02)]:
        f = o.bloom_build(np.array([h], np.uint64), 16, 1)
        bits = f[o.BLOOM_HDR:]
        assert bits[byte] == mask and sum(bits) == mask


def test_header_layout():
    f = o.bloom_build(_h([b"a"]), 64, 3)
    assert f[:4] == b"LSM\x03" and f[4] == 0 and f[5] == 0  # magic, StandardBloom, hash type 0
    assert int.from_bytes(f[6:14], "little") == 64 and int.from_bytes(f[14:22], "little") == 3
    assert len(f) == o.BLOOM_HDR + 8
    assert o.bloom_contains(b"XSM\x03" + f[4:], 0) == -1


def test_serde_round_trip_members():
    keys = [b"item%d" % i for i in range(10)]
    m, k = o.bloom_shape(10, fpr=0.0001)
    f = o.bloom_build(_h(keys), m, k)
    for key in keys:
        assert o.bloom_contains(f, o.xxh3_64(key)) == 1
    for absent in (b"asdasads", b"item10", b"cxycxycxy", b"asdasdasdasdasdasdasd"):
        assert o.bloom_contains(f, o.xxh3_64(absent)) == 0


@pytest.mark.parametrize("policy,n,lo,hi", [
    (("bpk", 5.0), 1_000, 0.0, 0.13),
    (("fpr", 0.1), 100_000, 0.05, 0.13),
    (("fpr", 0.5), 100_000, 0.45, 0.55),
])
def test_false_positive_bands(policy, n, lo, hi):
    kw = {policy[0]: policy[1]}
    m, k = o.bloom_shape(n, **kw)
    f = o.bloom_build(_h(_nanoids(n, 1)), m, k)
    probes = _h(_nanoids(n, 2))
    fp = sum(o.bloom_contains(f, int(h)) for h in probes) / n
    assert lo < fp < hi


def test_hash64_matches_python_xxhash():
    xxhash = pytest.importorskip("xxhash")
    for key in _nanoids(50, 3) + [b"", b"a", b"x" * 300]:
        assert o.xxh3_64(key) == xxhash.xxh3_64_intdigest(key)
