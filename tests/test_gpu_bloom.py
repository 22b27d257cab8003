"""GPU parity of the standard Bloom filter (lsm_hash64_keys, lsm_bloom_build,
lsm_bloom_contains) against the oracle's restatement (oracle/bloom.c) of
src/table/filter/standard_bloom/{builder,mod}.rs and bit_array/.
Bar: bit-exact filter images (header + bit array), identical contains answers,
hash64 identical to the oracle's xxh3_64 for every key-length class."""
import random

import numpy as np
import pytest

import pyoracle

pytestmark = pytest.mark.gpu


def _keys_to_device(gpu, keys):
    import torch
    off = np.zeros(len(keys) + 1, np.int64)
    off[1:] = np.cumsum([len(k) for k in keys])
    arena = b"".join(keys)
    return (gpu.to_device_bytes(np.frombuffer(arena, np.uint8) if arena else np.zeros(0, np.uint8)),
            torch.from_numpy(off).cuda())


def _u64(t):
    return t.cpu().numpy().view(np.uint64)


def test_hash64_keys_all_length_classes(gpu):
    r = random.Random(5)
    lens = [0, 1, 2, 3, 4, 5, 8, 9, 16, 17, 31, 128, 129, 200, 240, 241, 300, 1024, 1500] + \
           [r.randrange(1, 64) for _ in range(500)]
    keys = [bytes(r.randrange(256) for _ in range(n)) for n in lens]
    arena, off = _keys_to_device(gpu, keys)
    got = _u64(gpu.hash64_keys(arena, off))
    exp = np.array([pyoracle.xxh3_64(k) for k in keys], np.uint64)
    assert (got == exp).all()


@pytest.mark.parametrize("n,policy", [(1, ("bpk", 10.0)), (10, ("fpr", 0.0001)), (1000, ("bpk", 5.0)),
                                      (4097, ("bpk", 10.0)), (20000, ("fpr", 0.1)), (20000, ("fpr", 0.5))])
def test_bloom_build_bit_exact(gpu, n, policy):
    import torch
    rng = np.random.default_rng(n)
    hashes = rng.integers(0, 2 ** 63, n, dtype=np.int64).view(np.uint64) * np.uint64(2) + np.uint64(1)
    m, k = gpu.bloom_shape(n, **{policy[0]: policy[1]})
    assert (m, k) == pyoracle.bloom_shape(n, **{policy[0]: policy[1]})
    filt = gpu.bloom_build(torch.from_numpy(hashes.view(np.int64)).cuda(), m, k)
    exp = pyoracle.bloom_build(hashes, m, k)
    assert filt.cpu().numpy().tobytes() == exp
    probes = np.concatenate([hashes[: 2000], rng.integers(0, 2 ** 63, 3000, dtype=np.int64).view(np.uint64)])
    got = gpu.bloom_contains(filt, torch.from_numpy(probes.view(np.int64)).cuda()).cpu().numpy()
    assert (got[: min(n, 2000)] == 1).all()  # no false negatives
    assert list(got) == [pyoracle.bloom_contains(exp, int(h)) for h in probes]


def test_bloom_keys_end_to_end(gpu):
    """standard_bloom/mod.rs:127-203: item0..item9 at fpr 0.0001, members true, listed non-members false."""
    keys = [b"item%d" % i for i in range(10)]
    arena, off = _keys_to_device(gpu, keys)
    h = gpu.hash64_keys(arena, off)
    m, k = gpu.bloom_shape(10, fpr=0.0001)
    filt = gpu.bloom_build(h, m, k)
    assert filt.cpu().numpy().tobytes() == pyoracle.bloom_build(_u64(h), m, k)
    absent = [b"asdasads", b"item10", b"cxycxycxy", b"asdasdasdasdasdasdasd"]
    a2, o2 = _keys_to_device(gpu, keys + absent)
    got = gpu.bloom_contains(filt, gpu.hash64_keys(a2, o2)).cpu().numpy()
    assert list(got) == [1] * 10 + [0] * 4


def test_bloom_large_filter_property(gpu):
    """1M keys, BitsPerKey(10) (the writer default, filter/mod.rs:19-23): image equals the oracle's."""
    import torch
    n = 1 << 20
    rng = np.random.default_rng(1)
    hashes = rng.integers(0, 2 ** 63, n, dtype=np.int64).view(np.uint64) ^ np.uint64(1 << 63)
    m, k = gpu.bloom_shape(n, bpk=10.0)
    filt = gpu.bloom_build(torch.from_numpy(hashes.view(np.int64)).cuda(), m, k)
    assert filt.cpu().numpy().tobytes() == pyoracle.bloom_build(hashes, m, k)


def test_bloom_contains_bad_filter(gpu):
    import torch
    # BitsPerKey(0.5): m = n * (0.5 as usize) = 0; the reference panics in h1 % m, the ABI refuses
    m0, _ = gpu.bloom_shape(3, bpk=0.5)
    assert m0 == 0
    with pytest.raises(gpu.LsmError):
        gpu.bloom_build(torch.arange(1, 4, dtype=torch.int64).cuda(), m0, 1)
    m, k = gpu.bloom_shape(16, bpk=10.0)
    h = torch.arange(1, 9, dtype=torch.int64).cuda()
    filt = gpu.bloom_build(h, m, k).clone()
    filt[0] = ord("X")
    assert (gpu.bloom_contains(filt, h).cpu().numpy() == gpu.BLOOM_BAD_FILTER).all()
    good = gpu.bloom_build(h, m, k)
    assert (gpu.bloom_contains(good[:-1], h).cpu().numpy() == gpu.BLOOM_BAD_FILTER).all()  # truncated image
