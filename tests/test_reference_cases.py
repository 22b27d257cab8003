"""The oracle against the reference's OWN unit tests (tests/golden/reference_cases.json,
transcribed by tests/golden/make_reference_cases.py from the Rust asserts, one test id
per reference test name):
  src/table/data_block/mod.rs:565-1235       point_read, len, binary / hash index
  src/table/data_block/iter_test.rs:13-1280  forward iteration, seek / seek_upper ranges
  src/table/index_block/iter.rs:68-672       index block round trips
  src/table/block/hash_index/mod.rs:48-142   hash index bytes, conflicts, lookups
  src/table/block/header.rs:177-214          header round trip and corruption
The expectations are the reference's, not the oracle's: this pins the oracle (and,
in tests/test_gpu_reference_cases.py, the GPU) to the reference itself."""
import json
import struct
from pathlib import Path

import numpy as np
import pytest

import pyoracle

CASES = json.loads((Path(__file__).resolve().parent / "golden" / "reference_cases.json").read_text())
DATA = {c["name"]: c for c in CASES["data_block"]}
INDEX = {c["name"]: c for c in CASES["index_block"]}
HASH = {c["name"]: c for c in CASES["hash_index"]}
HEADER = {c["name"]: c for c in CASES["header"]}


def case_items(case):
    rows = [(bytes.fromhex(k), bytes.fromhex(v), s, t) for k, v, s, t in case["items"]]
    return pyoracle.Items.from_list(rows), rows


def trailer(payload):
    tr = payload[-31:]
    ri, step, bin_len, bin_off, hash_len, hash_off = struct.unpack_from("<BBIIII", tr, 0)
    return {"ri": ri, "bin_len": bin_len, "hash_len": hash_len, "item_count": struct.unpack_from("<I", tr, 27)[0]}


def check_data_case(case, payload, decoded, point_read, seek):
    """Every assertion of one reference data-block test against one encoded block.
    decoded: (n, parsed dict) of the block; point_read(needle, snap) -> index / -1;
    seek(lo, hi) -> (first, end, lo_found, hi_found)."""
    e = case["expect"]
    _, rows = case_items(case)
    tr = trailer(payload)
    n, parsed = decoded
    if "len" in e:
        assert tr["item_count"] == e["len"] and n == e["len"]
    if "count" in e:
        assert n == e["count"]
    if "binary_index_len" in e:
        assert tr["bin_len"] == e["binary_index_len"]
    if "hash_index" in e:
        assert (tr["hash_len"] > 0) == e["hash_index"]
    if e.get("forward"):
        got = pyoracle.materialize(payload, parsed, tr["ri"])
        assert len(got) == len(rows)
        for (gk, gv, gs, gt), (k, v, s, t) in zip(got, rows):
            assert (gk, gs, gt) == (k, s, t)  # InternalValue == compares (user_key, seqno), key.rs:14-18
            assert gv == (b"" if t in (1, 2) else v)  # tombstones carry no value (mod.rs:212-216)
    for needle, snap, want, tomb in e.get("point_reads", []):
        got = point_read(bytes.fromhex(needle), snap)
        assert got == (-1 if want is None else want), (needle, snap)
        if tomb is not None:
            assert (rows[got][3] in (1, 2)) == tomb
    for r in e.get("ranges", []):
        lo = None if r["lo"] is None else bytes.fromhex(r["lo"])
        hi = None if r["hi"] is None else bytes.fromhex(r["hi"])
        first, end, lo_found, hi_found = seek(lo, hi)
        a, b = r["range"]
        assert max(end - first, 0) == b - a and (b == a or first == a), (r, first, end)
        if r["lo_found"] is not None:
            assert lo_found == r["lo_found"]
        if r["hi_found"] is not None:
            assert hi_found == r["hi_found"]


def case_ris(case, cap=None):
    ris = case["restart_intervals"]
    return ris if cap is None or len(ris) <= cap else ris[:cap] + [ris[-1]]


@pytest.mark.parametrize("name", sorted(DATA))
def test_reference_data_block(name):
    case = DATA[name]
    items, _ = case_items(case)
    for ri in case_ris(case):
        payload = pyoracle.data_block_encode(items, restart_interval=ri, hash_ratio=case["hash_ratio"])
        blk = pyoracle.block_write(payload)
        assert pyoracle.block_verify(blk)[0] == 0
        n, parsed = pyoracle.data_block_decode(payload)
        check_data_case(case, payload, (n, parsed), lambda nd, sn: pyoracle.point_read(payload, nd, sn),
                        lambda lo, hi: pyoracle.seek(payload, lo, hi))


@pytest.mark.parametrize("name", sorted(INDEX))
def test_reference_index_block(name):
    case = INDEX[name]
    keys = [bytes.fromhex(k) for k, _, _, _ in case["items"]]
    it = pyoracle.Items.from_list([(k, b"", s, 0) for k, (_, s, _, _) in zip(keys, case["items"])])
    it.handle_off = np.array([o for _, _, o, _ in case["items"]], np.uint64)
    it.handle_size = np.array([z for _, _, _, z in case["items"]], np.uint32)
    payload = pyoracle.index_block_encode(it)
    n, parsed = pyoracle.data_block_decode(payload, index=True)
    assert n == case["expect"]["len"]
    for j, (k, s, o, z) in enumerate(case["items"]):  # KeyedBlockHandle == (end_key, seqno, handle)
        ko, kl = int(parsed["key_off"][j]), int(parsed["key_len"][j])
        assert payload[ko:ko + kl] == bytes.fromhex(k) and int(parsed["seqno"][j]) == s
        assert int(parsed["handle_off"][j]) == o and int(parsed["val_len"][j]) == z


@pytest.mark.parametrize("name", sorted(HASH))
def test_reference_hash_index(name):
    case = HASH[name]
    keys = [bytes.fromhex(k) for k, _ in case["sets"]]
    got = pyoracle.hash_index_build(keys, [i for _, i in case["sets"]], case["buckets"])
    assert list(got) == case["bytes"]
    assert sum(1 for b in got if b == 255) == case["conflicts"]
    for k, want in case["gets"]:
        assert pyoracle.hash_index_get(got, bytes.fromhex(k)) == want


@pytest.mark.parametrize("name", sorted(HEADER))
def test_reference_header(name):
    case = HEADER[name]
    hdr = bytearray(pyoracle.header_encode(case["block_type"], case["checksum"], case["data_length"],
                                           case["uncompressed_length"]))
    assert len(hdr) == 33  # Header::serialized_len
    if case["mutate_byte"] is not None:
        hdr[case["mutate_byte"]] = (hdr[case["mutate_byte"]] + 1) & 0xFF
    st, h = pyoracle.header_decode(bytes(hdr))
    want = {"OK": 0, "HDR_CKSUM": 3}[case["expect"]]
    assert st == want
    if st == 0:
        assert (h.block_type, h.cksum_lo, h.cksum_hi, h.data_length, h.uncompressed_length) == \
            (case["block_type"], case["checksum"], 0, case["data_length"], case["uncompressed_length"])
