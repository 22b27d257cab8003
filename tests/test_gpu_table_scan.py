"""Whole-table scan on the GPU: lsm_scan_table == Scanner
(src/table/scanner.rs:24-92) as restated by pyoracle.scanner, which reads the
data blocks back to back from offset 0 (Block::from_reader) and adds the
table's global_seqno to every item (:84).  The GPU walks the block index
instead (TLI -> [index partitions ->] data handles, block_index/full.rs,
two_level.rs), so agreement also checks that the index describes the same
blocks.  Tables come from pyoracle.table_write (writer/mod.rs:303-343,
writer/index/full.rs:55-69, writer/index/partitioned.rs:54-235)."""
import numpy as np
import pytest

from helpers import FIELD_VIEW, counter_items, prefix_items, random_sorted_items

pytestmark = pytest.mark.gpu


def _scan(L, t, global_seqno=0, block_count=None, cap_blocks=None, file=None, sync=True, hint=0, ihint=0):
    """sync=False: lsm_scan_table_async, its device results read back here and
    shaped like the synchronising call's (block_off cut to n_blocks + 1)."""
    import torch
    data = t["file"] if file is None else file
    d_file = L.to_device_bytes(data)
    bc = t["block_count"] if block_count is None else block_count
    out = L.scan_table(d_file, len(data), t["tli_off"], t["tli_size"], two_level=t.get("two_level", False),
                       global_seqno=global_seqno, block_count=bc, cap_blocks=cap_blocks, sync=sync,
                       data_blocks_hint=hint, index_blocks_hint=ihint)
    torch.cuda.synchronize()
    res = {k: (v.cpu().numpy() if hasattr(v, "cpu") else v) for k, v in out.items()}
    if not sync:
        res["table_status"] = int(res["table_status"][0])
        res["n_blocks"] = int(res["n_blocks"][0])
        res["block_off"] = res["block_off"][:res["n_blocks"] + 1]
    return res


def _table(oracle, items, two_level, **kw):
    t = oracle.table_write(items, two_level=two_level, **kw)
    t["two_level"] = two_level
    return t


def _check_against_scanner(oracle, g, t, global_seqno, data=None):
    """Blocks the oracle Scanner read before its first error must match; the first
    failing block must carry the Scanner's error status."""
    blocks, err = oracle.scanner(t["file"] if data is None else data, t["block_count"], global_seqno)
    assert g["table_status"] == 0
    nb = g["n_blocks"]
    assert nb == t["block_count"]
    assert (g["block_off"].view(np.uint64) == t["block_off"]).all()
    st = g["status"][:nb]
    starts = g["item_start"].view(np.uint32)
    for b, (pos, size, parsed) in enumerate(blocks):
        assert st[b] == 0, (b, st[b])
        assert int(g["block_off"][b]) == pos
        lo, hi = int(starts[b]), int(starts[b + 1])
        assert hi - lo == len(parsed["seqno"])
        for f, dt in FIELD_VIEW.items():
            if f == "handle_off":
                continue
            assert (g[f].view(dt)[lo:hi] == parsed[f].astype(dt)).all(), (b, f)
    if err:
        assert st[len(blocks)] == err, (len(blocks), st[len(blocks)], err)
    else:
        assert len(blocks) == nb and (st == 0).all()


@pytest.mark.parametrize("two_level", [False, True])
@pytest.mark.parametrize("global_seqno", [0, 7, 2 ** 64 - 10])
def test_scan_counter_table(gpu, oracle, two_level, global_seqno):
    t = _table(oracle, counter_items(52 * 300, seed=5, tomb_frac=0.05), two_level)
    g = _scan(gpu, t, global_seqno)
    _check_against_scanner(oracle, g, t, global_seqno)


@pytest.mark.parametrize("two_level", [False, True])
def test_scan_mixed_tables(gpu, oracle, two_level):
    for items, kw in ((random_sorted_items(3000, seed=3, big_seq=True), {"block_size": 1024}),
                      (prefix_items(56 * 40), {"block_size": 16384}),
                      (counter_items(820 * 6, seed=2), {"block_size": 65536}),
                      (random_sorted_items(400, seed=4), {"block_size": 64, "partition_size": 256})):
        t = _table(oracle, items, two_level, **kw)
        g = _scan(gpu, t, 3)
        _check_against_scanner(oracle, g, t, 3)


@pytest.mark.parametrize("two_level", [False, True])
def test_scan_many_blocks(gpu, oracle, two_level):
    # ~3000 data blocks: several decode workgroups per level, a TLI larger than the LDS stage
    t = _table(oracle, counter_items(52 * 3000, seed=8), two_level)
    g = _scan(gpu, t, 1)
    _check_against_scanner(oracle, g, t, 1)


def test_table_global_seqno_reference(gpu, oracle):
    """src/table/tests.rs:1379-1430 table_global_seqno: a0@0, a1@1, b@8, data block size 1,
    partitioned index with partition size 1, global_seqno 7 -> the table yields seqnos
    7, 8, 15 (a1 = 8 is invisible to snapshot 8)."""
    items = oracle.Items.from_list([(b"a0", b"a0", 0, 0), (b"a1", b"a1", 1, 0), (b"b", b"b", 8, 0)])
    t = _table(oracle, items, True, block_size=1, partition_size=1)
    assert t["block_count"] == 3
    g = _scan(gpu, t, 7)
    _check_against_scanner(oracle, g, t, 7)
    n = int(g["item_start"].view(np.uint32)[3])
    assert g["seqno"].view(np.uint64)[:n].tolist() == [7, 8, 15]


def test_table_return_global_seqno_reference(gpu, oracle):
    """src/table/tests.rs:1432-1470 table_return_global_seqno: abc@0 with global_seqno 15
    is returned as abc@15."""
    items = oracle.Items.from_list([(b"abc", b"abc", 0, 0)])
    t = _table(oracle, items, False)
    g = _scan(gpu, t, 15)
    _check_against_scanner(oracle, g, t, 15)
    assert int(g["seqno"].view(np.uint64)[0]) == 15 and int(g["key_len"].view(np.uint16)[0]) == 3


def test_scan_corrupt_data_block(gpu, oracle):
    t = _table(oracle, counter_items(52 * 50, seed=6), True)
    data = bytearray(t["file"])
    k = 17
    data[int(t["block_off"][k]) + 100] ^= 0x40  # payload byte -> checksum mismatch
    g = _scan(gpu, t, 0, file=bytes(data))
    _check_against_scanner(oracle, g, t, 0, data=bytes(data))
    assert g["status"][k] == 4  # CKSUM


def test_scan_table_level_errors(gpu, oracle):
    t = _table(oracle, counter_items(52 * 50, seed=6), False)
    # corrupt TLI payload -> its checksum status
    data = bytearray(t["file"])
    data[t["tli_off"] + 40] ^= 1
    assert _scan(gpu, t, file=bytes(data))["table_status"] == 4
    # metadata block count disagrees -> PARSE
    assert _scan(gpu, t, block_count=t["block_count"] + 1)["table_status"] == 5
    # more blocks than the caller's capacity -> OVERFLOW
    assert _scan(gpu, t, cap_blocks=10)["table_status"] == 6
    # TLI handle past the end of the file -> TRUNCATED
    bad = dict(t)
    bad["tli_size"] = t["tli_size"] + 1
    assert _scan(gpu, bad)["table_status"] == 8
    # handles that leave a gap (re-encoded TLI with a shifted data handle) -> TRUNCATED
    p = t["file"][t["tli_off"] + 33:t["tli_off"] + t["tli_size"]]
    n, parsed = oracle.data_block_decode(p, index=True)
    assert n == t["block_count"]
    offs = parsed["handle_off"].copy()
    offs[5] += 1
    keys = [p[int(a):int(a) + int(b)] for a, b in zip(parsed["key_off"], parsed["key_len"])]
    it = oracle.Items(np.frombuffer(b"".join(keys), np.uint8),
                      np.concatenate([[0], np.cumsum([len(k) for k in keys])]).astype(np.uint64),
                      np.zeros(0, np.uint8), np.zeros(n + 1, np.uint64), parsed["seqno"], np.zeros(n, np.uint8),
                      offs, parsed["val_len"])
    tli = oracle.block_write(oracle.index_block_encode(it), block_type=1)
    data = t["file"][:t["tli_off"]] + tli
    bad = dict(t)
    bad["tli_size"] = len(tli)
    assert _scan(gpu, bad, file=data)["table_status"] == 8
    # a data block as the TLI -> TYPE_MISMATCH (index expected)
    bad = dict(t)
    bad["tli_off"], bad["tli_size"] = 0, int(t["block_off"][1])
    assert _scan(gpu, bad)["table_status"] == 7


@pytest.mark.parametrize("two_level", [False, True])
def test_scan_async_matches(gpu, oracle, two_level):
    """lsm_scan_table_async (no host synchronisation, counts on the device): the
    same blocks, items and statuses as the Scanner, with a cap of about 4x the
    blocks and with the exact block count as the data hint."""
    t = _table(oracle, counter_items(52 * 600, seed=12, tomb_frac=0.05), two_level)
    for cap, hint, ihint in ((4 * t["block_count"], 0, 0), (4 * t["block_count"], t["block_count"],
                                                             t["tli_size"] // 4 if two_level else 0)):
        g = _scan(gpu, t, 9, cap_blocks=cap, sync=False, hint=hint, ihint=ihint)
        _check_against_scanner(oracle, g, t, 9)
    data = bytearray(t["file"])
    data[int(t["block_off"][23]) + 100] ^= 0x40
    g = _scan(gpu, t, 0, file=bytes(data), cap_blocks=2 * t["block_count"], sync=False)
    _check_against_scanner(oracle, g, t, 0, data=bytes(data))


def test_scan_async_level_errors(gpu, oracle):
    """The table statuses of test_scan_table_level_errors through the async call
    (n_blocks 0 for a failed table), plus a data hint below the block count."""
    t = _table(oracle, counter_items(52 * 50, seed=6), False)
    cap = 4 * t["block_count"]
    data = bytearray(t["file"])
    data[t["tli_off"] + 40] ^= 1
    g = _scan(gpu, t, file=bytes(data), cap_blocks=cap, sync=False)
    assert g["table_status"] == 4 and g["n_blocks"] == 0
    assert _scan(gpu, t, block_count=t["block_count"] + 1, cap_blocks=cap, sync=False)["table_status"] == 5
    assert _scan(gpu, t, cap_blocks=10, sync=False)["table_status"] == 6
    assert _scan(gpu, t, cap_blocks=cap, hint=t["block_count"] - 1, sync=False)["table_status"] == 6
    bad = dict(t)
    bad["tli_size"] = t["tli_size"] + 1
    assert _scan(gpu, bad, cap_blocks=cap, sync=False)["table_status"] == 8
    bad = dict(t)
    bad["tli_off"], bad["tli_size"] = 0, int(t["block_off"][1])
    assert _scan(gpu, bad, cap_blocks=cap, sync=False)["table_status"] == 7
    t2 = _table(oracle, counter_items(52 * 50, seed=6), True, partition_size=256)
    assert _scan(gpu, t2, cap_blocks=4 * t2["block_count"], sync=False)["table_status"] == 0
    assert _scan(gpu, t2, cap_blocks=4 * t2["block_count"], ihint=1, sync=False)["table_status"] == 6
