"""The C-ABI entry points captured into a HIP graph (torch.cuda.CUDAGraph over
the caller's stream) and replayed: lsm_encode_blocks with and without the
workspace pool (4 KiB blocks; an item-parallel-planned batch of group-class,
listed and 1 MiB blocks; a batch holding a ~3.7 MiB block, whose pool decode
streams its checksum chain inside the parse launch) and lsm_decode_blocks with
and without the pool.
Every replay's output == the oracle's (bytes, offsets, statuses, every
decoded field).  A graph replays the launches the capture recorded, so every
per-call clear must be a node that runs on each replay (csrc/fill.hpp)."""
import numpy as np
import pytest

import pyoracle
from helpers import compare_decode, counter_items

pytestmark = pytest.mark.gpu

BATCHES = {
    "4KiB": [52] * 300,
    "mixed": [50, 200, 20000, 7, 1, 30000, 300, 13, 9000, 64, 65, 129, 2500, 16400],
    # a ~3.7 MiB block (>= 64 windows of 32 KiB): with the pool the decode streams its XXH3
    # chain behind the parse units inside one launch (unit-done flags cleared per call)
    "streamed": [52, 52429, 3300, 52],
}


def _items(gpu, sizes, seed):
    import torch
    items = counter_items(int(sum(sizes)), seed=seed, tomb_frac=0.05)
    starts = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint32)
    d_items = gpu.items_to_device(items)
    d_starts = torch.from_numpy(starts.astype(np.int32)).cuda()
    return items, starts, d_items, d_starts


def _capture(fn):
    """fn() once on a side stream (allocations, LDS attributes), then captured."""
    import torch
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    return g


@pytest.mark.parametrize("pool", [True, False])
@pytest.mark.parametrize("batch", sorted(BATCHES))
def test_encode_graph_replay(gpu, batch, pool):
    import torch
    sizes = BATCHES[batch]
    items, starts, d_items, d_starts = _items(gpu, sizes, seed=17)
    nb = len(sizes)
    ref_buf, ref_off = pyoracle.encode_blocks(items, starts)
    enc = gpu.Encoder()
    out = enc.encode(d_items, d_starts, nb, pool=pool)
    graph = _capture(lambda: enc.encode(d_items, d_starts, nb, out=out, pool=pool))
    for _ in range(3):
        out["buf"].zero_()
        out["status"].fill_(-1)
        out["block_off"].fill_(-1)
        graph.replay()
        torch.cuda.synchronize()
        off = out["block_off"].cpu().numpy().view(np.uint64)
        assert (out["status"].cpu().numpy()[:nb] == 0).all() and (off == ref_off).all()
        assert out["buf"].cpu().numpy()[:int(off[-1])].tobytes() == ref_buf.tobytes()


@pytest.mark.parametrize("sizes", [[52] * 300, [205] * 120], ids=["4KiB-asked", "16KiB-auto"])
def test_encode_graph_replay_run_plan(gpu, sizes):
    """The run-level plan in the group kernel (LSM_ENCODE_RUN_PLAN, or by itself at >= 128
    items per block): its look-back words are cleared by a kernel node on every replay."""
    import torch
    items, starts, d_items, d_starts = _items(gpu, sizes, seed=29)
    nb = len(sizes)
    ref_buf, ref_off = pyoracle.encode_blocks(items, starts)
    enc = gpu.Encoder()
    out = enc.encode(d_items, d_starts, nb, pool=False, run_plan=True)
    graph = _capture(lambda: enc.encode(d_items, d_starts, nb, out=out, pool=False, run_plan=True))
    for _ in range(3):
        out["buf"].zero_()
        out["status"].fill_(-1)
        out["block_off"].fill_(-1)
        graph.replay()
        torch.cuda.synchronize()
        off = out["block_off"].cpu().numpy().view(np.uint64)
        assert (out["status"].cpu().numpy()[:nb] == 0).all() and (off == ref_off).all()
        assert out["buf"].cpu().numpy()[:int(off[-1])].tobytes() == ref_buf.tobytes()


@pytest.mark.parametrize("pool", [True, False])
@pytest.mark.parametrize("batch", sorted(BATCHES))
def test_decode_graph_replay(gpu, batch, pool):
    import torch
    sizes = BATCHES[batch]
    items, starts, _, _ = _items(gpu, sizes, seed=23)
    buf, off = pyoracle.encode_blocks(items, starts)
    buf = bytearray(buf)
    buf[int(off[1]) + 40] ^= 0x10  # block 1: payload checksum mismatch
    buf = np.frombuffer(bytes(buf), np.uint8)
    parsed, item_start, status = pyoracle.decode_blocks(buf, off)
    assert status[1] == 4
    nb = len(off) - 1
    d_blocks = gpu.to_device_bytes(buf)
    d_off = torch.from_numpy(off.astype(np.int64)).cuda()
    n_cap = len(buf) // 3 + 1
    dec = gpu.Decoder()
    out = dec.alloc_outputs(n_cap, nb)
    graph = _capture(lambda: dec.decode(d_blocks, d_off, nb, out, n_cap, pool=pool))
    for _ in range(3):
        for v in out.values():
            v.fill_(-1)
        graph.replay()
        torch.cuda.synchronize()
        g = {k: v.cpu().numpy() for k, v in out.items()}
        g["status"] = g["status"][:nb]
        compare_decode(g, parsed, item_start, status)
