"""Data blocks above the general path's 72 KiB stage, up to the writer's 4 MiB
data-block target (use_data_block_size, src/table/writer/mod.rs:193-198):
encoded on the device (E3, straight in HBM) bit-exact against the oracle and
decoded through the stage in 64 KiB chunks (decode_chunked: per-KiB XXH3
contributions on all waves, the chain carried across chunks, intervals parsed
from LDS or walked from HBM when they straddle the staged window).
Cases: 256 KiB, 1 MiB and 4 MiB blocks, hash ratio 0 and 1.33 (the hash index
is dropped above 254 restart heads, trailer.rs:100-111), restart intervals 16
and 1, tombstones, a flipped payload bit (CKSUM) and a broken record re-sealed
with valid checksums (PARSE).  Bar: bit-exact bytes, statuses and fields."""
import numpy as np
import pytest

import pyoracle
from helpers import compare_decode, counter_items, gpu_decode, pack

pytestmark = pytest.mark.gpu


def _gpu_encode(gpu, items, starts, ri, ratio):
    import torch
    d_items = gpu.items_to_device(items)
    d_starts = torch.from_numpy(np.asarray(starts, np.int64).astype(np.int32)).cuda()
    out = gpu.Encoder().encode(d_items, d_starts, len(starts) - 1, restart_interval=ri, hash_ratio=ratio)
    torch.cuda.synchronize()
    off = out["block_off"].cpu().numpy().view(np.uint64)
    return out["buf"].cpu().numpy()[:int(off[-1])], off, out["status"].cpu().numpy()[:len(starts) - 1]


@pytest.mark.parametrize("ratio", [0.0, 1.33])
@pytest.mark.parametrize("ri", [16, 1])
def test_large_data_blocks_round_trip(gpu, ri, ratio):
    items = counter_items(80000, seed=41 + ri, tomb_frac=0.05)
    starts = np.array([0, 3300, 16400, 78200, 80000], np.uint32)  # ~256 KiB, 1 MiB, 4 MiB, ~130 KiB blocks
    ref_buf, ref_off = pyoracle.encode_blocks(items, starts, restart_interval=ri, hash_ratio=ratio)
    sizes = np.diff(ref_off.astype(np.int64))
    assert sizes.max() > 4_100_000 and (sizes > 72 * 1024).all(), sizes
    buf, off, st = _gpu_encode(gpu, items, starts, ri, ratio)
    assert (st == 0).all() and (off == ref_off).all() and buf.tobytes() == ref_buf.tobytes()
    g = gpu_decode(gpu, buf, off)
    parsed, item_start, status = pyoracle.decode_blocks(buf, off)
    assert (status == 0).all()
    compare_decode(g, parsed, item_start, status)


def test_large_data_blocks_corrupted(gpu):
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
    g = gpu_decode(gpu, buf2, off2)
    parsed, item_start, status = pyoracle.decode_blocks(buf2, off2)
    assert (status[:2] == 0).all() and status[2] == 4 and (status[3:] != 0).all(), status
    compare_decode(g, parsed, item_start, status)


@pytest.mark.parametrize("ratio", [0.0, 1.33])
def test_large_blocks_few_items(gpu, ratio):
    """Blocks beyond the 96 KiB list image with at most 256 items (long values):
    E3 takes their record offsets from its own workgroup scan (E1 keeps full
    32-bit offsets only for blocks of more than 256 items); long seqnos and
    value lengths give multi-byte varints."""
    items = counter_items(400, key_len=24, val_len=3000, seqno=(1 << 40) + 5, seed=11, tomb_frac=0.1)
    starts = np.array([0, 40, 290, 400], np.uint32)  # ~110 KiB, ~680 KiB (250 items), ~300 KiB
    ref_buf, ref_off = pyoracle.encode_blocks(items, starts, restart_interval=16, hash_ratio=ratio)
    sizes = np.diff(ref_off.astype(np.int64))
    assert (sizes > 96 * 1024).all(), sizes
    buf, off, st = _gpu_encode(gpu, items, starts, 16, ratio)
    assert (st == 0).all() and (off == ref_off).all() and buf.tobytes() == ref_buf.tobytes()
    g = gpu_decode(gpu, buf, off)
    parsed, item_start, status = pyoracle.decode_blocks(buf, off)
    assert (status == 0).all()
    compare_decode(g, parsed, item_start, status)
