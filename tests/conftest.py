import json
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
for p in (ROOT, ROOT / "oracle", ROOT / "lsm-tree_amd"):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))

GOLDEN = Path(__file__).resolve().parent / "golden"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C ABI)")
    config.addinivalue_line("markers", "slow: longer CPU cases")


@pytest.fixture(scope="session")
def golden_blocks():
    return json.loads((GOLDEN / "blocks.json").read_text())["cases"]


@pytest.fixture(scope="session")
def xxh3_kat():
    return json.loads((GOLDEN / "xxh3_kat.json").read_text())["vectors"]


@pytest.fixture(scope="session")
def oracle():
    import pyoracle
    pyoracle.lib()
    return pyoracle


def case_items(case):
    """Golden JSON case -> pyoracle.Items."""
    import numpy as np
    import pyoracle
    if case["kind"] == "index":
        rows = [(bytes.fromhex(k), int(s), int(o), int(sz)) for k, s, o, sz in case["items"]]
        keys = b"".join(r[0] for r in rows)
        kl = np.array([len(r[0]) for r in rows], np.uint64)
        key_off = np.concatenate([[0], np.cumsum(kl)]).astype(np.uint64)
        n = len(rows)
        return pyoracle.Items(np.frombuffer(keys, np.uint8), key_off, np.zeros(1, np.uint8), np.zeros(n + 1, np.uint64),
                              np.array([r[1] for r in rows], np.uint64), np.zeros(n, np.uint8),
                              np.array([r[2] for r in rows], np.uint64), np.array([r[3] for r in rows], np.uint32))
    rows = [(bytes.fromhex(k), bytes.fromhex(v), int(s), int(t)) for k, v, s, t in case["items"]]
    return pyoracle.Items.from_list(rows)


def case_expected_items(case):
    """Expected materialized items for a case (what DataBlock::iter + materialize yields)."""
    if case["kind"] == "index":
        return [(bytes.fromhex(k), int(s), int(o), int(sz)) for k, s, o, sz in case["items"]]
    return [(bytes.fromhex(k), b"" if int(t) in (1, 2) else bytes.fromhex(v), int(s), int(t))
            for k, v, s, t in case["items"]]


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import lsmgpu
    lsmgpu.lib()
    return lsmgpu


@pytest.fixture(scope="session")
def diag_lib(gpu):
    """The diagnostic build (lsm-tree_amd/.variants/libdiag.so, -DLSM_DIAG: the flag bits
    that force the guard paths), loaded beside the product library with the same ctypes
    signatures; tests swap it in for one call."""
    from pathlib import Path
    path = Path(gpu.HERE) / ".variants" / "libdiag.so"
    if not path.exists():
        pytest.fail(f"{path} not built (__graft_entry__.build() builds the diagnostic variant)")
    saved, saved_path = gpu._lib, gpu.LIB_PATH
    gpu._lib, gpu.LIB_PATH = None, path
    try:
        lib = gpu.lib()
    finally:
        gpu._lib, gpu.LIB_PATH = saved, saved_path
    return lib
