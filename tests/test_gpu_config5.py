"""configs[4]-shaped mixed batch on the GPU, checked block by block against the
oracle: equal bytes of 4/16/64 KiB data blocks with G1 (counter) and G2
(random sorted) keys, each segment followed by its index blocks (restart
interval 1, one per 64 MiB table: writer/mod.rs:284-290,
index_block/block_handle.rs:134-156), in ONE buffer.  The batch is decoded
whole and as two byte-balanced shards (lsmgpu.shard_blocks),
and every status, item_start and parsed field (handle_off included) must equal
pyoracle.decode_blocks.  bench.build_config5_shard also memcmp-checks every
GPU-encoded data and index block against pyoracle.encode_blocks."""
import os
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

pytestmark = pytest.mark.gpu

THREADS = min(16, os.cpu_count() or 1)


def test_config5_mixed_batch_whole_and_sharded(gpu):
    import torch

    import bench
    lsmgpu = gpu
    blocks, boff, nb, n_items, nbytes, n_idx, checked = bench.build_config5_shard(torch, lsmgpu, 96 << 20, 0,
                                                                                 THREADS)
    assert n_idx >= 6 and checked == nb
    host = blocks[:nbytes].cpu().numpy()
    hoff = boff.cpu().numpy().view(np.uint64)
    fields = bench.DATA_FIELDS + ["handle_off"]
    # whole batch
    _, out = bench.time_decode(torch, lsmgpu, blocks, boff, nb, n_items, 1, fields=fields)
    n_all = bench.check_decode_all(out, host, hoff, nb, THREADS, fields=fields)
    assert n_all == n_items
    # two byte-balanced shards of the same buffer (block_off stays absolute)
    bounds = lsmgpu.shard_blocks(hoff, 2)
    assert bounds[0] == 0 and bounds[-1] == nb and 0 < bounds[1] < nb
    sizes = [int(hoff[bounds[r + 1]] - hoff[bounds[r]]) for r in range(2)]
    assert abs(sizes[0] - sizes[1]) <= 70000  # one 64 KiB block at most
    n_sum = 0
    for r in range(2):
        b0, b1 = bounds[r], bounds[r + 1]
        sb = b1 - b0
        sub_off = boff[b0:b1 + 1]
        cap = int(n_items)
        dec = lsmgpu.Decoder(blocks.device)
        so = dec.alloc_outputs(cap, sb, fields=fields)
        dec.decode(blocks, sub_off, sb, so, cap)
        torch.cuda.synchronize()
        n_sum += bench.check_decode_all(so, host, np.ascontiguousarray(hoff[b0:b1 + 1]), sb, THREADS, fields=fields)
    assert n_sum == n_items
