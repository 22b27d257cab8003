"""Encode argument checks on the device: block ranges the C ABI must vet
because the reference's types guarantee them (DataBlock::encode_into takes
&[InternalValue], src/table/data_block/mod.rs:523-549).  A block whose item
range runs past n_items, is empty, or holds an over-long key (key_off going
backwards) gets LSM_BAD_ARG and zero bytes; every other block stays
bit-exact with the oracle encoding of that block alone."""
import numpy as np
import pytest

import pyoracle
from helpers import counter_items, random_sorted_items

pytestmark = pytest.mark.gpu

BAD_ARG = 10


def _encode(gpu, items, starts, ri, ratio):
    import torch
    d_items = gpu.items_to_device(items)
    d_starts = torch.from_numpy(np.asarray(starts, np.int64).astype(np.uint32).view(np.int32)).cuda()
    out = gpu.Encoder().encode(d_items, d_starts, len(starts) - 1, restart_interval=ri, hash_ratio=ratio)
    torch.cuda.synchronize()
    off = out["block_off"].cpu().numpy().view(np.uint64)
    buf = out["buf"].cpu().numpy()[:int(off[-1])]
    return buf, off, out["status"].cpu().numpy()[:len(starts) - 1]


def _check(items, starts, buf, off, st, bad, ri, ratio):
    nb = len(starts) - 1
    for b in range(nb):
        if b in bad:
            assert st[b] == BAD_ARG, (b, st[b])
            assert off[b + 1] == off[b], b
            continue
        assert st[b] == 0, (b, st[b])
        ref, _ = pyoracle.encode_blocks(items, np.array([starts[b], starts[b + 1]], np.uint32),
                                        restart_interval=ri, hash_ratio=ratio)
        assert buf[int(off[b]):int(off[b + 1])].tobytes() == ref.tobytes(), b


@pytest.mark.parametrize("ratio", [0.0, 1.33])
def test_encode_starts_past_n_items(gpu, ratio):
    """starts[n] and an interior start past n_items (monotone): those blocks
    are BAD_ARG, the blocks before them bit-exact; an empty block in the middle
    is BAD_ARG and the blocks after it stay good."""
    items = counter_items(3000, seed=21)
    n = items.n
    good = list(range(0, 2900, 52))           # blocks of 52 items
    starts = good + [n + 3, n + 40]           # (2860, n+3) and (n+3, n+40) run past n_items
    starts[10] = starts[9]                    # block 9 empty
    starts = np.array(starts, np.int64)
    buf, off, st = _encode(gpu, items, starts, 16, ratio)
    nb = len(starts) - 1
    _check(items, starts, buf, off, st, {9, nb - 2, nb - 1}, 16, ratio)


@pytest.mark.parametrize("ratio", [0.0, 1.33])
def test_encode_backward_key_offsets(gpu, ratio):
    """key_off going backwards inside one block (at hash ratio > 0 with keys
    longer than 16 bytes, which the bucket fixup kernel hashes): that block is
    BAD_ARG, nothing reads the ~4 GiB 'key', the other blocks are bit-exact."""
    items = random_sorted_items(1200, seed=31, kmin=17, kmax=60, vmax=40)
    starts = np.array(list(range(0, 1200, 40)) + [1200], np.int64)
    ko = items.key_off.copy()
    i = 205                                   # inside block 5 = items [200, 240)
    ko[i + 1] = ko[i] - 1                     # item i's key length wraps to ~2^64
    bad_items = pyoracle.Items(items.keys, ko, items.vals, items.val_off, items.seqno, items.vtype)
    buf, off, st = _encode(gpu, bad_items, starts, 4, ratio)
    # blocks other than 5 only use offsets of their own items, unchanged
    _check(items, starts, buf, off, st, {5}, 4, ratio)


@pytest.mark.parametrize("ratio", [0.0, 1.33])
def test_encode_huge_batch_args(gpu, ratio):
    """A batch of ~20 Ki items per block (the item-parallel plan, E1p): a
    40 000-item block, an empty one, a 50-item one, a 59 950-item one and one
    past n_items: the empty and the out-of-range blocks are BAD_ARG, the others
    bit-exact."""
    items = counter_items(100000, seed=23)
    starts = np.array([0, 40000, 40000, 40050, 99000 + 1000, 100005], np.int64)
    starts[4] = 100000 - 1000  # (block 3: 58 950 items)
    buf, off, st = _encode(gpu, items, starts, 16, ratio)
    _check(items, starts, buf, off, st, {1, 4}, 16, ratio)


def test_encode_huge_batch_not_monotone(gpu):
    """E1p: an item_start array that goes backwards rejects every block."""
    items = counter_items(100000, seed=24)
    starts = np.array([0, 40000, 30000, 100000], np.int64)
    _, off, st = _encode(gpu, items, starts, 16, 0.0)
    assert (st == BAD_ARG).all(), st
    assert (off == 0).all()
