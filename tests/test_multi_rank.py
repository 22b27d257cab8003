"""N > 1 path on CPU: world_size-2 gloo ranks shard a block batch by bytes
(lsmgpu.shard_blocks), each rank decodes only its shard
(oracle decode as the per-rank worker, since there is no GPU here), and the
gathered per-rank results equal one decode of the whole batch.  No
collective touches the data path except this test's final check."""
import os
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parent.parent
for p in (ROOT / "lsm-tree_amd", ROOT / "oracle", ROOT / "tests"):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))

import lsmgpu  # noqa: E402
import pyoracle  # noqa: E402
from helpers import random_sorted_items  # noqa: E402


def _batch():
    items = random_sorted_items(3000, seed=31)
    starts = pyoracle.cut_blocks(items, 1024)
    return pyoracle.encode_blocks(items, starts, restart_interval=4)


def _worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    buf, off = _batch()
    bounds = lsmgpu.shard_blocks(off, world)
    b0, b1 = bounds[rank], bounds[rank + 1]
    sub_off = off[b0:b1 + 1] - off[b0]
    sub = buf[int(off[b0]):int(off[b1])].copy()
    parsed, item_start, status = pyoracle.decode_blocks(sub, sub_off)
    mine = torch.from_numpy(np.concatenate([status.astype(np.int64), parsed["seqno"][:int(item_start[-1])].view(np.int64)]))
    sizes = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(sizes, torch.tensor([mine.numel()]))
    mx = int(max(s.item() for s in sizes))
    padded = torch.zeros(mx, dtype=torch.int64)
    padded[:mine.numel()] = mine
    got = [torch.zeros(mx, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(got, padded)
    if rank == 0:
        q.put([g[:int(s.item())].numpy() for g, s in zip(got, sizes)] + [bounds])
    dist.barrier()
    dist.destroy_process_group()


def test_shard_blocks_bounds():
    off = np.array([0, 10, 20, 1000, 1010, 1020], np.uint64)
    b = lsmgpu.shard_blocks(off, 2)
    assert b[0] == 0 and b[-1] == 5 and b == sorted(b)
    assert lsmgpu.shard_blocks(off, 1) == [0, 5]
    assert lsmgpu.shard_blocks(np.array([0], np.uint64), 4) == [0, 0, 0, 0, 0]
    eq = np.arange(0, 801, 100, dtype=np.uint64)  # 8 equal blocks
    assert lsmgpu.shard_blocks(eq, 4) == [0, 2, 4, 6, 8]


@pytest.mark.timeout(300)
def test_two_rank_gloo_shards_cover_batch():
    import multiprocessing as mp
    import socket
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = q.get(timeout=240)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    parts, bounds = res[:2], res[2]
    buf, off = _batch()
    parsed, item_start, status = pyoracle.decode_blocks(buf, off)
    n = len(off) - 1
    assert bounds[0] == 0 and bounds[-1] == n and 0 < bounds[1] < n
    st = np.concatenate([parts[r][:bounds[r + 1] - bounds[r]] for r in range(2)])
    seq = np.concatenate([parts[r][bounds[r + 1] - bounds[r]:] for r in range(2)])
    assert (st == status).all()
    assert (seq.view(np.uint64) == parsed["seqno"][:int(item_start[-1])]).all()


def test_shard_items_cuts_at_blocks_and_balances_bytes():
    """Encode-side split: block-aligned, about equal key + value bytes."""
    import numpy as np
    import lsmgpu
    rng = np.random.default_rng(3)
    per_block = rng.integers(1, 200, 997)
    starts = np.concatenate([[0], np.cumsum(per_block)]).astype(np.int64)
    n_items = int(starts[-1])
    kl = rng.integers(1, 64, n_items).astype(np.uint64)
    vl = rng.integers(0, 512, n_items).astype(np.uint64)
    ko = np.concatenate([[0], np.cumsum(kl)]).astype(np.uint64)
    vo = np.concatenate([[0], np.cumsum(vl)]).astype(np.uint64)
    for world in (1, 2, 3, 8):
        b = lsmgpu.shard_items(starts, ko, vo, world)
        assert len(b) == world + 1 and b[0] == 0 and b[-1] == len(per_block)
        assert all(x <= y for x, y in zip(b, b[1:]))
        w = ko[starts] + vo[starts]
        sizes = [int(w[b[r + 1]] - w[b[r]]) for r in range(world)]
        blk = np.diff(w.astype(np.int64))
        assert max(sizes) - min(sizes) <= 2 * int(blk.max())
