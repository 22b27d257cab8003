"""Host-side checks of the ctypes mirror's workspace handling (no GPU: the
library is replaced by a recorder; the size functions are the real ones).

Since ABI 7 the huge-block pool is an explicit opt-in (LSM_DECODE_HUGE_POOL /
LSM_ENCODE_HUGE_POOL, include/lsmgpu.h): a pool=True call passes the flag and
the _ex workspace, a pool=False call neither.  A Decoder reused across calls
still hands a pool=False call exactly lsm_decode_workspace_size(n), however
large an earlier pool=True call grew its cached buffer."""
import ctypes as C

import pytest
import torch

import lsmgpu


class _Recorder:
    def __init__(self, real):
        self.real = real
        self.calls = []

    def __getattr__(self, name):
        if name.startswith("lsm_decode_workspace_size") or name.startswith("lsm_encode_workspace_size") \
                or name == "lsm_encode_bound":
            return getattr(self.real, name)

        def rec(*args):
            self.calls.append((name, args))
            return 0
        return rec


@pytest.fixture
def fake(monkeypatch):
    real = lsmgpu.lib()
    r = _Recorder(real)
    monkeypatch.setattr(lsmgpu, "lib", lambda: r)
    monkeypatch.setattr(lsmgpu, "_torch", lambda: torch)
    monkeypatch.setattr(lsmgpu, "_stream", lambda s: C.c_void_p(0))
    return r


def _ws_arg(call):
    name, args = call
    assert name in ("lsm_decode_blocks", "lsm_decode_blocks_tuned")
    return args[9], args[8]  # workspace_bytes, workspace pointer


def _pool_flag(call):
    name, args = call
    if name == "lsm_decode_blocks":  # (no tuning: never the pool)
        return False
    return bool(args[10]._obj.flags & lsmgpu.DECODE_HUGE_POOL)


def test_decoder_pool_then_no_pool(fake):
    n = 100
    blocks = torch.zeros(n * 300 * 1024, dtype=torch.uint8)  # 300 KiB mean: the pool would pay
    off = torch.zeros(n + 1, dtype=torch.int64)
    d = lsmgpu.Decoder("cpu")
    out = d.alloc_outputs(16, n)
    d.decode(blocks, off, n, out, 16, pool=True)
    d.decode(blocks, off, n, out, 16, pool=False)
    d.decode(blocks, off, n, out, 16)  # default: the mean block size picks the pool
    base = fake.real.lsm_decode_workspace_size(n)
    full = fake.real.lsm_decode_workspace_size_ex(n, blocks.numel())
    got = [_ws_arg(c)[0] for c in fake.calls]
    assert got == [full, base, full]
    assert [_pool_flag(c) for c in fake.calls] == [True, False, True]
    threshold = ((base + 255) & ~255) + 8704  # lsmgpu.h: the pool threshold
    assert base < threshold <= full
    # the cached buffer is reused (one allocation), only its view changes
    assert len({_ws_arg(c)[1].value for c in fake.calls}) == 1


def test_encoder_passes_exact_workspace(fake):
    n_items, n_blocks = 64, 4
    items = {"keys": torch.zeros(64 * 16 + 64, dtype=torch.uint8),
             "key_off": torch.arange(n_items + 1, dtype=torch.int64) * 16,
             "vals": torch.zeros(64 * 64 + 64, dtype=torch.uint8),
             "val_off": torch.arange(n_items + 1, dtype=torch.int64) * 64,
             "seqno": torch.zeros(n_items, dtype=torch.int64), "vtype": torch.zeros(n_items, dtype=torch.uint8)}
    starts = torch.arange(0, n_items + 1, 16, dtype=torch.int32)
    e = lsmgpu.Encoder("cpu")
    e.encode(items, starts, n_blocks, pool=True)
    e.encode(items, starts, n_blocks, pool=False)
    ws = [args[9] for name, args in fake.calls if name == "lsm_encode_blocks"]
    assert ws[1] == fake.real.lsm_encode_workspace_size(n_items, n_blocks) < ws[0]
    flags = [args[3]._obj.flags for name, args in fake.calls if name == "lsm_encode_blocks"]
    assert flags == [lsmgpu.ENCODE_HUGE_POOL, 0]


def test_encoder_run_plan_flag(fake):
    """run_plan=True asks for the run-level plan (LSM_ENCODE_RUN_PLAN), alone or with the pool."""
    n_items, n_blocks = 64, 4
    items = {"keys": torch.zeros(64 * 16 + 64, dtype=torch.uint8),
             "key_off": torch.arange(n_items + 1, dtype=torch.int32) * 16,
             "vals": torch.zeros(64 * 64 + 64, dtype=torch.uint8),
             "val_off": torch.arange(n_items + 1, dtype=torch.int32) * 64,
             "seqno": torch.zeros(n_items, dtype=torch.int64), "vtype": torch.zeros(n_items, dtype=torch.uint8)}
    starts = torch.arange(0, n_items + 1, 16, dtype=torch.int32)
    e = lsmgpu.Encoder("cpu")
    e.encode(items, starts, n_blocks, pool=False, run_plan=True)
    e.encode(items, starts, n_blocks, pool=True, run_plan=True)
    e.encode(items, starts, n_blocks, pool=False)
    calls = [(name, args) for name, args in fake.calls if name.startswith("lsm_encode_blocks")]
    assert [name for name, _ in calls] == ["lsm_encode_blocks32"] * 3  # (int32 offsets: the u32 entry)
    assert [args[3]._obj.flags for _, args in calls] == [lsmgpu.ENCODE_RUN_PLAN,
                                                         lsmgpu.ENCODE_HUGE_POOL | lsmgpu.ENCODE_RUN_PLAN, 0]
