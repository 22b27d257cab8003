"""CPU tests of the C-ABI library: it loads, exports every entry point declared
in include/lsmgpu.h, and its host-only helpers agree with the oracle.  No
device compute here (no GPU in this container)."""
import re
import random
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parent.parent


@pytest.fixture(scope="module")
def L():
    import lsmgpu
    if not lsmgpu.LIB_PATH.exists():
        lsmgpu.build()
    return lsmgpu


def declared_functions():
    text = (ROOT / "include" / "lsmgpu.h").read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(lsm_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_expected_entry_points():
    fns = declared_functions()
    for f in ("lsm_decode_blocks", "lsm_encode_blocks", "lsm_cut_blocks", "lsm_xxh3_128_batch",
              "lsm_decode_workspace_size", "lsm_encode_workspace_size", "lsm_encode_bound"):
        assert f in fns


def test_library_exports_every_declared_symbol(L):
    lib = L.lib()
    for f in declared_functions():
        assert hasattr(lib, f), f"{f} declared in include/lsmgpu.h but not exported"
    assert set(declared_functions()) == set(L.EXPORTED_SYMBOLS)


def test_library_exports_exactly_the_header(L):
    """nm -D of the product library lists the header's functions and nothing else
    (no diagnostic entry points, no C++ internals)."""
    import subprocess
    out = subprocess.run(["nm", "-D", "--defined-only", str(L.LIB_PATH)], check=True, capture_output=True,
                         text=True).stdout
    syms = {line.split()[-1] for line in out.splitlines() if line.strip()}
    syms = {s for s in syms if not s.startswith("_init") and not s.startswith("_fini")}
    assert syms == set(declared_functions())


def test_abi_version_and_status_names(L):
    lib = L.lib()
    assert lib.lsm_abi_version() == L.ABI_VERSION == 7
    for code, name in L.STATUS.items():
        assert lib.lsm_status_name(code).decode() == name


def test_cut_blocks_matches_oracle(L, oracle):
    rng = random.Random(11)
    for _ in range(30):
        n = rng.randint(1, 400)
        rows = [(b"k" * rng.randint(1, 40), b"v" * rng.randint(0, 300), 0, 0) for _ in range(n)]
        it = oracle.Items.from_list(rows)
        bs = rng.choice([1, 64, 512, 4096, 16384])
        assert list(L.cut_blocks(it.key_off, it.val_off, bs)) == list(oracle.cut_blocks(it, bs))


def test_encode_bound_covers_oracle_sizes(L, oracle):
    import ctypes as C
    rng = random.Random(5)
    for ri, ratio in ((1, 0.0), (16, 0.0), (4, 1.33), (1, 8.0)):
        rows = []
        for i in range(300):
            rows.append((i.to_bytes(8, "big") * rng.randint(1, 5), b"x" * rng.randint(0, 200), rng.getrandbits(63),
                         rng.choice([0, 1, 2, 4])))
        it = oracle.Items.from_list(rows)
        starts = oracle.cut_blocks(it, 2048)
        blocks, off = oracle.encode_blocks(it, starts, restart_interval=ri, hash_ratio=ratio, nthreads=2)
        p = L.LsmBlockParams(ri, 0, 0, 0, ratio)
        bound = L.lib().lsm_encode_bound(it.n, len(starts) - 1, len(it.keys), len(it.vals), C.byref(p))
        assert bound >= int(off[-1])


def test_workspace_sizes_monotone(L):
    lib = L.lib()
    assert lib.lsm_decode_workspace_size(1) <= lib.lsm_decode_workspace_size(1 << 20)
    assert lib.lsm_encode_workspace_size(10, 1) <= lib.lsm_encode_workspace_size(10 << 20, 1 << 18)


def test_bad_args_rejected_without_device(L):
    """Argument validation happens before any HIP call."""
    import ctypes as C
    lib = L.lib()
    ps = L.LsmParsed()
    # NULL buffers
    assert lib.lsm_decode_blocks(None, None, 4, -1, C.byref(ps), 10, None, None, None, 0, None) == 10
    # misaligned block buffer
    assert lib.lsm_decode_blocks(C.c_void_p(0x1001), C.c_void_p(0x2000), 4, -1, C.byref(ps), 10,
                                 C.c_void_p(0x3000), C.c_void_p(0x4000), C.c_void_p(0x5000), 1 << 20, None) == 10
    # n_blocks == 0 is a no-op
    assert lib.lsm_decode_blocks(None, None, 0, -1, C.byref(ps), 10, None, None, None, 0, None) == 0
    it = L.LsmItems()
    p = L.LsmBlockParams(16, 0, 1, 0, 0.0)  # LZ4 compression not supported
    assert lib.lsm_encode_blocks(C.byref(it), C.c_void_p(8), 1, C.byref(p), C.c_void_p(16), 100, C.c_void_p(24),
                                 C.c_void_p(32), C.c_void_p(48), 1 << 20, None) == 9
    p = L.LsmBlockParams(0, 0, 0, 0, 0.0)   # restart interval 0 (encoder.rs:91 divides by it)
    assert lib.lsm_encode_blocks(C.byref(it), C.c_void_p(8), 1, C.byref(p), C.c_void_p(16), 100, C.c_void_p(24),
                                 C.c_void_p(32), C.c_void_p(48), 1 << 20, None) == 10
    p = L.LsmBlockParams(16, 0, 0, 0, -1.0)  # negative hash ratio (builder.rs:40 asserts)
    assert lib.lsm_encode_blocks(C.byref(it), C.c_void_p(8), 1, C.byref(p), C.c_void_p(16), 100, C.c_void_p(24),
                                 C.c_void_p(32), C.c_void_p(48), 1 << 20, None) == 10
    for bits in (1, 2, 4, 0x80):  # lsm_block_params.reserved must be 0 (diagnostic ablations are not in the release)
        p = L.LsmBlockParams(16, 0, 0, bits, 0.0)
        assert lib.lsm_encode_blocks(C.byref(it), C.c_void_p(8), 1, C.byref(p), C.c_void_p(16), 100, C.c_void_p(24),
                                     C.c_void_p(32), C.c_void_p(48), 1 << 20, None) == 10
    for flags in (4, 8, 0x100, 1 << 31):  # lsm_block_params.flags: only LSM_ENCODE_HUGE_POOL | LSM_ENCODE_RUN_PLAN
        p = L.LsmBlockParams(16, 0, 0, 0, 0.0, flags)
        assert lib.lsm_encode_blocks(C.byref(it), C.c_void_p(8), 1, C.byref(p), C.c_void_p(16), 100, C.c_void_p(24),
                                     C.c_void_p(32), C.c_void_p(48), 1 << 20, None) == 10


def test_decode_tuning_flags_rejected(L):
    """Only LSM_DECODE_ITEM_START_VALID, LSM_DECODE_PAYLOAD_VERIFIED and
    LSM_DECODE_HUGE_POOL are public decode flags: diagnostic bits that would
    skip the hash, the parse or the stores, or force the streamed chains to
    give up, are LSM_BAD_ARG."""
    import ctypes as C
    lib = L.lib()
    ps = L.LsmParsed()
    ws = lib.lsm_decode_workspace_size(4)
    for flags in (8, 0x100, 0x200, 0x400, 0x800, 0x1000, 0x2000, 0x4000, 0x8000, 0x10000, 0x80000, 1 << 31):
        t = L.LsmDecodeTuning(0, 0, 0, flags)
        assert lib.lsm_decode_blocks_tuned(C.c_void_p(0x1000), C.c_void_p(0x2000), 4, -1, C.byref(ps), 10,
                                           C.c_void_p(0x3000), C.c_void_p(0x4000), C.c_void_p(0x5000), ws,
                                           C.byref(t), None) == 10
    for bad in ((64, 0, 0, 0), (0, 128, 0, 0), (0, 1 << 17, 0, 0), (0, 0, 9000, 0)):
        t = L.LsmDecodeTuning(*bad)
        assert lib.lsm_decode_blocks_tuned(C.c_void_p(0x1000), C.c_void_p(0x2000), 4, -1, C.byref(ps), 10,
                                           C.c_void_p(0x3000), C.c_void_p(0x4000), C.c_void_p(0x5000), ws,
                                           C.byref(t), None) == 10


def test_point_read_rejects_misaligned_buffers(L):
    import ctypes as C
    lib = L.lib()
    res = L.LsmPointResult(C.c_void_p(0x9000), None, None, None, None)
    args = [C.c_void_p(0x1000), C.c_void_p(0x2000), 4, C.c_void_p(0x3000), C.c_void_p(0x4000), C.c_void_p(0x5000),
            C.c_void_p(0x6000), 8, C.byref(res), C.c_void_p(0x7000), None]
    for i in (0, 4):  # d_blocks, d_needles
        a = list(args)
        a[i] = C.c_void_p(0x1000 + 8 * (i + 1))
        assert lib.lsm_point_read_blocks(*a) == 10


def test_product_path_has_no_cpu_fallback(L):
    """Without a GPU the product refuses to run instead of silently using a CPU path."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(L.LsmError):
        L.decode_blocks(torch.zeros(128, dtype=torch.uint8), torch.zeros(2, dtype=torch.int64))


def test_bench_workload_cut_rules(L):
    """The fixed item counts bench.py cuts its synthetic batches at equal the
    reference writer rule (writer/mod.rs:284-290) for every BASELINE shape
    (52 @ 4 KiB 16/64, 56 @ 16 KiB 40/256, 205 @ 16 KiB,
    820 @ 64 KiB)."""
    import sys
    sys.path.insert(0, str(ROOT))
    import bench
    for ipb, kl, vl, bs in ((52, 16, 64, 4096), (56, 40, 256, 16384), (205, 16, 64, 16384), (820, 16, 64, 65536)):
        bench.check_cut_rule(L, ipb, kl, vl, bs)
    for bs, ipb, kind, est in bench.C5_SEGMENTS:
        bench.check_cut_rule(L, ipb, 16, 64, bs)


@pytest.mark.parametrize("n,kw", [(1000, {"fpr": 0.01}), (1000, {"fpr": 0.1}), (1_000_000, {"fpr": 0.1}),
                                  (10, {"fpr": 0.0001}), (10, {"fpr": 0.0}), (1_000_000, {"bpk": 10.0}),
                                  (3, {"bpk": 5.0}), (7, {"bpk": 0.5}), (100_000, {"fpr": 0.5})])
def test_bloom_shape_matches_oracle(L, oracle, n, kw):
    assert L.bloom_shape(n, **kw) == oracle.bloom_shape(n, **kw)


def test_bloom_calculate_m_kats(L):
    lib = L.lib()  # standard_bloom/builder.rs:173-187
    assert [lib.lsm_bloom_calculate_m(1000, 0.01), lib.lsm_bloom_calculate_m(1000, 0.1),
            lib.lsm_bloom_calculate_m(1_000_000, 0.1)] == [9_592, 4_800, 4_792_536]
    with pytest.raises(L.LsmError):
        L.bloom_shape(0, bpk=10.0)
