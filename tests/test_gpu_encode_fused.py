"""The run-level plan fused into the encode group kernel (encode_group_kernel<..., true>):
each 32-block run plans its own blocks and takes its output offset from the runs before it
by a decoupled look-back (csrc/encode.hip run_lookback), with no plan launch and no size
scan.  Taken for data blocks without a hash index, <= 512 items per block on average, no
pool, when asked for (LSM_ENCODE_RUN_PLAN, as here) or at >= 128 items per block.  Every case is bit-exact against the oracle (DataBlock::encode_into +
Block::write_into, src/table/data_block/mod.rs:523-549, src/table/block/mod.rs:45-84),
through lsm_encode_blocks32 and lsm_encode_blocks, and checks that the fused path ran (every
run's look-back word holds an inclusive prefix)."""
import ctypes as C
import random

import numpy as np
import pytest

import pyoracle
from helpers import counter_items, random_sorted_items

pytestmark = pytest.mark.gpu

RUN = 32                 # kGRun
DIAG_LOOKBACK_GIVE_UP = 0x20


def _al256(x):
    return (x + 255) // 256 * 256


def _encode(gpu, items, starts, off32, ri=16, reserved=0, lib=None):
    import torch
    d = gpu.items_to_device(items, off32=off32)
    nb = len(starts) - 1
    d_starts = torch.from_numpy(np.asarray(starts, np.int64).astype(np.int32)).cuda()
    L = lib or gpu.lib()
    it = gpu.LsmItems32() if off32 else gpu.LsmItems()
    it.keys, it.key_off = d["keys"].data_ptr(), d["key_off"].data_ptr()
    it.vals, it.val_off = d["vals"].data_ptr(), d["val_off"].data_ptr()
    it.seqno, it.vtype = d["seqno"].data_ptr(), d["vtype"].data_ptr()
    it.n_items = d["seqno"].numel()
    params = gpu.LsmBlockParams(ri, 0, 0, reserved, 0.0, gpu.ENCODE_RUN_PLAN)
    bound = L.lsm_encode_bound(it.n_items, nb, d["keys"].numel(), d["vals"].numel(), C.byref(params))
    need = L.lsm_encode_workspace_size(it.n_items, nb)
    ws = torch.zeros(max(need, 256), dtype=torch.uint8, device="cuda")
    buf = torch.zeros(bound + gpu.LSM_INPUT_PADDING, dtype=torch.uint8, device="cuda")
    off = torch.zeros(nb + 1, dtype=torch.int64, device="cuda")
    st = torch.full((max(nb, 1),), -1, dtype=torch.int32, device="cuda")
    fn = L.lsm_encode_blocks32 if off32 else L.lsm_encode_blocks
    rc = fn(C.byref(it), C.c_void_p(d_starts.data_ptr()), nb, C.byref(params), C.c_void_p(buf.data_ptr()), bound,
            C.c_void_p(off.data_ptr()), C.c_void_p(st.data_ptr()), C.c_void_p(ws.data_ptr()), need, None)
    assert rc == 0, rc
    torch.cuda.synchronize()
    o = off.cpu().numpy().view(np.uint64)
    # the look-back words (the workspace's sizes array on this path, encode.hip launch_encode)
    runs = (nb + RUN - 1) // RUN
    base = 2 * _al256((nb + 1) * 8)
    lb = ws[base:base + 8 * runs].cpu().numpy().view(np.uint64)
    return buf.cpu().numpy(), o, st.cpu().numpy()[:nb], lb


def _check(gpu, items, starts, ri=16):
    ref_buf, ref_off = pyoracle.encode_blocks(items, starts, restart_interval=ri)
    for off32 in (True, False):
        buf, off, st, lb = _encode(gpu, items, starts, off32, ri=ri)
        assert (st == 0).all(), (off32, np.flatnonzero(st)[:10], st[st != 0][:10])
        assert (off == ref_off).all(), off32
        assert buf[:int(off[-1])].tobytes() == ref_buf.tobytes(), off32
        assert ((lb >> np.uint64(62)) == 2).all(), "the fused path did not run (look-back words)"
        assert ((lb & np.uint64((1 << 40) - 1)) <= off[-1]).all()


@pytest.mark.parametrize("nb", [1, 31, 32, 33, 65, 250])
def test_fused_run_boundaries(gpu, nb):
    """Batches ending inside, at and past a run; random 1-120 item blocks over restart intervals."""
    rng = random.Random(nb)
    sizes = [rng.randint(1, 120) for _ in range(nb)]
    items = random_sorted_items(sum(sizes), seed=nb + 5, vmax=120)
    starts = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint32)
    _check(gpu, items, starts, ri=rng.choice([1, 4, 16]))


def test_fused_mixed_classes(gpu):
    """Group-class blocks with listed ones (medium / big list kernels, one-workgroup E3) in
    the same runs: the fused kernel numbers the listed blocks for the list kernels."""
    items = random_sorted_items(12000, seed=77, kmax=40, vmax=700, big_seq=True)
    rng = random.Random(3)
    starts = [0]
    while starts[-1] < items.n:
        want = rng.choice([2, 20, 40, 60, 150, 400]) if rng.random() < 0.3 else rng.randint(1, 12)
        starts.append(min(items.n, starts[-1] + want))
    assert (items.n / (len(starts) - 1)) <= 512
    _check(gpu, items, np.array(starts, np.uint32))


def test_fused_many_runs(gpu):
    """625 runs (the look-back walks windows of 64 runs at the start of the grid)."""
    items = counter_items(52 * 20000, seed=11, tomb_frac=0.01)
    starts = np.arange(0, 52 * 20000 + 1, 52, dtype=np.uint32)
    _check(gpu, items, starts)


def test_fused_rejected_block(gpu):
    """A start array that goes backwards: LSM_BAD_ARG for the blocks planned with the
    offending ones (here the 32-block run that holds them, include/lsmgpu.h), no bytes
    for them, and every other block as the oracle encodes it."""
    items = counter_items(52 * 100, seed=2)
    starts = np.arange(0, 52 * 100 + 1, 52, dtype=np.uint32)
    bad = starts.copy()
    bad[40] = bad[41] + 1  # block 39 ends after block 40 starts, block 40 runs backwards
    buf, off, st, lb = _encode(gpu, items, bad, True)
    assert (st[RUN:2 * RUN] == 10).all(), st[RUN:2 * RUN]
    assert (off[RUN:2 * RUN + 1] == off[RUN]).all()
    assert ((lb >> np.uint64(62)) == 2).all()
    for b in list(range(RUN)) + list(range(2 * RUN, 100)):
        assert st[b] == 0, (b, st[b])
        ref, _ = pyoracle.encode_blocks(items, np.array([bad[b], bad[b + 1]], np.uint32))
        assert buf[int(off[b]):int(off[b + 1])].tobytes() == ref.tobytes(), b


def test_fused_give_up(gpu, diag_lib):
    """Diagnostic build, reserved bit 0x20: every run but the first gives up its look-back at
    once.  Run 0's blocks are encoded as the oracle's; every block of a later run reports
    LSM_INCOMPLETE (13), none a success with bytes at an unknown offset."""
    items = counter_items(52 * 100, seed=4)
    starts = np.arange(0, 52 * 100 + 1, 52, dtype=np.uint32)
    ref_buf, ref_off = pyoracle.encode_blocks(items, starts)
    buf, off, st, lb = _encode(gpu, items, starts, True, reserved=DIAG_LOOKBACK_GIVE_UP, lib=diag_lib)
    assert (st[:RUN] == 0).all(), st[:RUN]
    assert (st[RUN:] == 13).all(), st[RUN:]
    end0 = int(ref_off[RUN])
    assert (off[:RUN] == ref_off[:RUN]).all()
    assert buf[:end0].tobytes() == ref_buf[:end0].tobytes()
    assert (lb[1:] >> np.uint64(61) & np.uint64(1)).all(), "later runs publish poison"
    # the same library without the flag: as the release
    buf2, off2, st2, _ = _encode(gpu, items, starts, True, lib=diag_lib)
    assert (st2 == 0).all() and (off2 == ref_off).all() and buf2[:int(off2[-1])].tobytes() == ref_buf.tobytes()


def test_fused_concurrent_streams(gpu):
    """Two batches encoded with the run-level plan on two streams at once (each call its own
    workspace and look-back words): both bit-exact."""
    import torch
    a_items = counter_items(205 * 300, seed=31)
    b_items = random_sorted_items(9000, seed=32, vmax=120)
    a_starts = np.arange(0, 205 * 300 + 1, 205, dtype=np.uint32)
    rng = random.Random(5)
    b_starts = [0]
    while b_starts[-1] < b_items.n:
        b_starts.append(min(b_items.n, b_starts[-1] + rng.randint(1, 120)))
    b_starts = np.array(b_starts, np.uint32)
    outs = []
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    encs = [gpu.Encoder(), gpu.Encoder()]
    jobs = [(a_items, a_starts), (b_items, b_starts)]
    dev = []
    for items, starts in jobs:
        d = gpu.items_to_device(items, off32=True)
        ds = torch.from_numpy(starts.astype(np.int32)).cuda()
        dev.append((d, ds, len(starts) - 1))
    torch.cuda.synchronize()
    for (d, ds, nb), s, e in zip(dev, streams, encs):
        with torch.cuda.stream(s):
            outs.append(e.encode(d, ds, nb, pool=False, run_plan=True, stream=s))
    torch.cuda.synchronize()
    for (items, starts), out in zip(jobs, outs):
        nb = len(starts) - 1
        ref_buf, ref_off = pyoracle.encode_blocks(items, starts)
        off = out["block_off"].cpu().numpy().view(np.uint64)
        assert (out["status"].cpu().numpy()[:nb] == 0).all() and (off == ref_off).all()
        assert out["buf"].cpu().numpy()[:int(off[-1])].tobytes() == ref_buf.tobytes()
