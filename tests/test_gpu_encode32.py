"""lsm_encode_blocks32: the encode over lsm_items32 (u32 key / value offsets,
SURVEY §8(d)'s 4 + 4 bytes per item) runs the same kernels as
lsm_encode_blocks with the offset arrays read 4 bytes wide.  Every case here
is encoded both ways and compared bit for bit with the oracle
(DataBlock::encode_into + Block::write_into, src/table/data_block/mod.rs:523-549,
src/table/block/mod.rs:45-84): random batches over restart intervals and hash
ratios, every size class (group, medium / big list kernels, E3, the pool's
whole-GPU E3 with E1p planning), index blocks, the configs[1] shape."""
import random

import numpy as np
import pytest

import pyoracle
from helpers import counter_items, index_items, random_sorted_items

pytestmark = pytest.mark.gpu


def _encode(gpu, items, starts, off32, ri=16, ratio=0.0, block_type=0, pool=None):
    import torch
    d_items = gpu.items_to_device(items, off32=off32)
    assert d_items["key_off"].element_size() == (4 if off32 else 8)
    d_starts = torch.from_numpy(np.asarray(starts, np.int64).astype(np.int32)).cuda()
    out = gpu.Encoder().encode(d_items, d_starts, len(starts) - 1, restart_interval=ri, hash_ratio=ratio,
                               block_type=block_type, pool=pool)
    torch.cuda.synchronize()
    off = out["block_off"].cpu().numpy().view(np.uint64)
    return out["buf"].cpu().numpy()[:int(off[-1])].tobytes(), off, out["status"].cpu().numpy()[:len(starts) - 1]


def _check(gpu, items, starts, **kw):
    ref_buf, ref_off = pyoracle.encode_blocks(items, starts, restart_interval=kw.get("ri", 16),
                                              hash_ratio=kw.get("ratio", 0.0), block_type=kw.get("block_type", 0))
    for off32 in (True, False):
        buf, off, st = _encode(gpu, items, starts, off32, **kw)
        assert (st == 0).all(), (off32, st)
        assert (off == ref_off).all(), off32
        assert buf == ref_buf.tobytes(), off32


@pytest.mark.parametrize("ri", [1, 5, 16])
@pytest.mark.parametrize("ratio", [0.0, 1.33])
def test_encode32_random_batches(gpu, ri, ratio):
    items = random_sorted_items(3000, seed=ri * 11 + int(ratio), vmax=120)
    rng = random.Random(ri + 3)
    starts = [0]
    while starts[-1] < items.n:
        starts.append(min(items.n, starts[-1] + rng.randint(1, 120)))
    _check(gpu, items, np.array(starts, np.uint32), ri=ri, ratio=ratio)


@pytest.mark.parametrize("ratio", [0.0, 1.33])
def test_encode32_size_classes(gpu, ratio):
    """Group, medium and big list kernels and the one-workgroup E3 (blocks up to ~250 KiB)."""
    items = random_sorted_items(1500, seed=int(ratio * 100) + 9, kmax=40, vmax=700, big_seq=True)
    starts = [0]
    for want in (3, 40, 9, 150, 1, 400, 25, 60, 700, 2, 110):
        starts.append(min(items.n, starts[-1] + want))
    if starts[-1] < items.n:
        starts.append(items.n)
    _check(gpu, items, np.array(starts, np.uint32), ratio=ratio)


@pytest.mark.parametrize("pool", [True, False])
def test_encode32_large_blocks(gpu, pool):
    """~256 KiB, 1 MiB and 4 MiB blocks: E1p (item-parallel plan) and, with the
    pool, the whole-GPU E3 (record units, chains)."""
    items = counter_items(80000, seed=43, tomb_frac=0.05)
    starts = np.array([0, 3300, 16400, 78200, 80000], np.uint32)
    _check(gpu, items, starts, pool=pool)


def test_encode32_index_blocks(gpu):
    items = index_items(2000)
    starts = np.array(list(range(0, 2000, 97)) + [2000], np.uint32)
    _check(gpu, items, starts, ri=1, block_type=1)


def test_encode32_config1_shape(gpu):
    """The headline shape (16 B keys, 64 B values, 52 items per 4 KiB block)."""
    items = counter_items(52 * 2048, seed=5)
    starts = np.arange(0, 52 * 2048 + 1, 52, dtype=np.uint32)
    _check(gpu, items, starts)


def test_encode32_argument_checks(gpu):
    import ctypes as C
    lib = gpu.lib()
    it = gpu.LsmItems32()
    it.n_items = 4
    p = gpu.LsmBlockParams(16, 0, 0, 0, 0.0, 0)
    # NULL key_off
    assert lib.lsm_encode_blocks32(C.byref(it), C.c_void_p(8), 1, C.byref(p), C.c_void_p(16), 100, C.c_void_p(24),
                                   C.c_void_p(32), C.c_void_p(48), 1 << 20, None) == 10
    it.key_off = 64
    it.val_off = 64
    it.n_items = 0xFFFFFFFF  # u32 offsets index n_items + 1 entries
    assert lib.lsm_encode_blocks32(C.byref(it), C.c_void_p(8), 1, C.byref(p), C.c_void_p(16), 100, C.c_void_p(24),
                                   C.c_void_p(32), C.c_void_p(48), 1 << 20, None) == 10
