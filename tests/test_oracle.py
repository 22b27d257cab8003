"""CPU tests: pin the oracle (oracle/, test infrastructure) to the reference's
known answers and the committed golden vectors.

Reference tests mirrored (fjall-rs/lsm-tree 3.1.9):
  src/hash.rs:11-32                         hash KATs
  src/table/block/hash_index/mod.rs:48-142  hash-index bytes & conflict rules
  src/table/block/header.rs:177-214         header round trip / corruption
  src/table/block/mod.rs:192-230            block round trip
  src/table/data_block/mod.rs:565-1235      point reads (subset, semantic)
  src/table/writer/mod.rs:547-587           chunk accounting
"""
import random

import numpy as np
import pytest

from conftest import case_expected_items, case_items


def test_hash_kats(oracle):
    assert oracle.xxh3_64(bytes([0, 0, 0])) == 16_959_823_422_411_450_475
    assert oracle.xxh3_64(bytes([0, 0, 1])) == 8_004_557_073_989_523_290
    assert oracle.xxh3_128(bytes([0, 0, 0])) == 321_827_061_816_535_117_015_859_907_874_601_773_163
    assert oracle.xxh3_128(bytes([0, 0, 1])) == 154_036_699_985_066_753_773_347_827_765_470_844_762


def test_xxh3_golden_vectors(oracle, xxh3_kat):
    for v in xxh3_kat:
        n = v["len"]
        b = bytes(((31 * i + 7) & 0xFF) for i in range(n))
        assert oracle.xxh3_64(b) == int(v["xxh3_64"]), n
        assert oracle.xxh3_128(b) == int(v["xxh3_128"]), n


def test_xxh3_vs_python_xxhash(oracle):
    xxhash = pytest.importorskip("xxhash")
    rng = random.Random(7)
    for n in list(range(0, 600)) + [rng.randint(600, 20000) for _ in range(50)]:
        b = bytes(rng.getrandbits(8) for _ in range(n))
        assert oracle.xxh3_64(b) == xxhash.xxh3_64_intdigest(b), n
        assert oracle.xxh3_128(b) == xxhash.xxh3_128_intdigest(b), n


def test_hash_index_kat_positions(oracle):
    # hash_index/mod.rs:49-79: buckets for "a","b","c" mod 100 are 19, 15, 11
    assert oracle.xxh3_64(b"a") % 100 == 19
    assert oracle.xxh3_64(b"b") % 100 == 15
    assert oracle.xxh3_64(b"c") % 100 == 11


def test_appendix_b_block(oracle):
    items = oracle.Items.from_list([(b"pla:earth:fact", b"eaaaaaaaaarth", 0, 0)])
    payload = oracle.data_block_encode(items, restart_interval=16, hash_ratio=0.0)
    assert payload.hex() == ("00000e706c613a65617274683a666163740d65616161616161616161727468ff0000"
                             "10020100000020000000000000000000000001000000000000000001000000")
    blk = oracle.block_write(payload)
    assert blk[:33].hex() == "4c534d0300de4adbc6de9c817fcd96c0742a6fb32b4100000041000000e742de23"


def test_golden_blocks_encode(oracle, golden_blocks):
    for case in golden_blocks:
        items = case_items(case)
        if case["kind"] == "index":
            payload = oracle.index_block_encode(items)
        else:
            payload = oracle.data_block_encode(items, restart_interval=case["restart_interval"],
                                               hash_ratio=case["hash_ratio"])
        blk = oracle.block_write(payload, case["block_type"])
        assert blk.hex() == case["block"], case["name"]


def test_golden_blocks_decode(oracle, golden_blocks):
    for case in golden_blocks:
        blk = bytes.fromhex(case["block"])
        st, h = oracle.block_verify(blk)
        assert st == 0, case["name"]
        assert h.block_type == case["block_type"]
        payload = blk[33:]
        n, parsed = oracle.data_block_decode(payload, index=case["kind"] == "index")
        assert n == len(case["items"]), case["name"]
        if case["kind"] == "index":
            exp = case_expected_items(case)
            for i, (k, s, o, sz) in enumerate(exp):
                ko, kl = int(parsed["key_off"][i]), int(parsed["key_len"][i])
                assert payload[ko:ko + kl] == k
                assert int(parsed["seqno"][i]) == s
                assert int(parsed["handle_off"][i]) == o
                assert int(parsed["val_len"][i]) == sz
        else:
            got = oracle.materialize(payload, parsed, case["restart_interval"])
            assert got == case_expected_items(case), case["name"]


def test_header_roundtrip_and_corruption(oracle):
    # header.rs:177-214 — flipping byte 5 (first checksum byte) -> ChecksumMismatch
    blk = oracle.block_write(b"abcdefabcdefabcdef", 0)
    st, h = oracle.header_decode(blk)
    assert st == 0 and h.data_length == 18 and h.uncompressed_length == 18
    bad = bytearray(blk)
    bad[5] = (bad[5] + 1) & 0xFF
    assert oracle.header_decode(bytes(bad))[0] == 3  # HDR_CKSUM
    bad = bytearray(blk)
    bad[0] = ord("X")
    assert oracle.header_decode(bytes(bad))[0] == 1  # BAD_MAGIC
    bad = bytearray(blk)
    bad[4] = 9
    assert oracle.header_decode(bytes(bad))[0] == 2  # BAD_TYPE (checked before the header checksum)
    bad = bytearray(blk)
    bad[40] ^= 1
    assert oracle.block_verify(bytes(bad))[0] == 4   # payload CKSUM
    assert oracle.header_decode(blk[:20])[0] == 8    # TRUNCATED


def test_block_roundtrip_uncompressed(oracle):
    # block/mod.rs:192-209
    blk = oracle.block_write(b"abcdefabcdefabcdef", 0)
    st, h = oracle.block_verify(blk)
    assert st == 0 and blk[33:] == b"abcdefabcdefabcdef"


def _sorted_items(rng, n, vt_choices=(0, 1, 2, 4)):
    raw = {}
    for _ in range(n):
        k = bytes(rng.choice(b"abcd") for _ in range(rng.randint(1, 10)))
        s = rng.randint(0, 50)
        t = rng.choice(vt_choices)
        v = b"" if t in (1, 2) else bytes(rng.getrandbits(8) for _ in range(rng.randint(0, 30)))
        raw[(k, s)] = (v, t)
    keys = sorted(raw, key=lambda ks: (ks[0], -ks[1]))
    return [(k, raw[(k, s)][0], s, raw[(k, s)][1]) for k, s in keys]


@pytest.mark.parametrize("ri", [1, 2, 3, 4, 7, 16])
@pytest.mark.parametrize("ratio", [0.0, 1.0, 1.33])
def test_fuzz_properties(oracle, ri, ratio):
    """fuzz/data_block/src/main.rs:130-323 properties (seeded): len, hash-index
    presence, full materialisation, every point_read."""
    rng = random.Random(ri * 1000 + int(ratio * 100))
    for _ in range(20):
        items = _sorted_items(rng, rng.randint(1, 80))
        it = oracle.Items.from_list(items)
        payload = oracle.data_block_encode(it, restart_interval=ri, hash_ratio=ratio)
        n, parsed = oracle.data_block_decode(payload)
        assert n == len(items)
        got = oracle.materialize(payload, parsed, ri)
        assert got == [(k, b"" if t in (1, 2) else v, s, t) for k, v, s, t in items]
        bin_len = int.from_bytes(payload[-31 + 2:-31 + 6], "little")
        hash_len = int.from_bytes(payload[-31 + 10:-31 + 14], "little")
        if bin_len > 254:
            assert hash_len == 0
        elif ratio > 0:
            assert hash_len > 0
        # point reads: the newest version visible at snapshot seqno+1 is the item itself
        for idx, (k, v, s, t) in enumerate(items):
            got_idx = oracle.point_read(payload, k, s + 1)
            exp = next(j for j, (k2, _, s2, _) in enumerate(items) if k2 == k and s2 < s + 1)
            assert got_idx == exp, (idx, k, s)
        assert oracle.point_read(payload, b"zzzzzzzzzzzz", 1 << 62) == -1


def test_point_read_mvcc(oracle):
    # data_block/mod.rs:581-640 style: MVCC shadowing, snapshot excludes >= seqno
    items = [(b"a", b"a3", 3, 0), (b"a", b"a2", 2, 0), (b"a", b"a1", 1, 0), (b"b", b"", 5, 1), (b"c", b"c", 0, 0)]
    for ri in range(1, 6):
        for ratio in (0.0, 1.33):
            payload = oracle.data_block_encode(oracle.Items.from_list(items), restart_interval=ri, hash_ratio=ratio)
            assert oracle.point_read(payload, b"a", 1 << 63) == 0
            assert oracle.point_read(payload, b"a", 3) == 1
            assert oracle.point_read(payload, b"a", 2) == 2
            assert oracle.point_read(payload, b"a", 1) == -1
            assert oracle.point_read(payload, b"b", 6) == 3
            assert oracle.point_read(payload, b"c", 1) == 4
            assert oracle.point_read(payload, b"d", 1) == -1
            assert oracle.point_read(payload, b"", 1) == -1


def test_writer_chunking(oracle):
    # writer/mod.rs:547-587: chunk_size += key.len() + value.len(); spill at >= block size
    it = oracle.Items.from_list([(b"a", b"a", 0, 0), (b"b", b"b", 0, 0), (b"c", b"c", 0, 0)])
    assert list(oracle.cut_blocks(it, 4)) == [0, 2, 3]
    assert list(oracle.cut_blocks(it, 1)) == [0, 1, 2, 3]
    assert list(oracle.cut_blocks(it, 1000)) == [0, 3]
    # BASELINE config 1: 16 B keys / 64 B values, 4 KiB -> 52 items per block
    n = 52 * 3
    items = [(i.to_bytes(16, "big"), b"\x00" * 64, 63, 0) for i in range(n)]
    starts = oracle.cut_blocks(oracle.Items.from_list(items), 4096)
    assert list(starts) == [0, 52, 104, 156]


def test_batch_encode_decode_roundtrip(oracle):
    rng = random.Random(3)
    items = [(i.to_bytes(16, "big"), bytes(rng.getrandbits(8) for _ in range(64)), 63, 0) for i in range(52 * 40)]
    it = oracle.Items.from_list(items)
    starts = oracle.cut_blocks(it, 4096)
    blocks, off = oracle.encode_blocks(it, starts, nthreads=4)
    # config 1 shape: 3769 B on disk per block; a restart interval
    # that crosses a 256-multiple of the BE counter shares one byte less per item
    sizes = np.diff(off.astype(np.int64))
    assert sizes[0] == 3769 and sizes.min() == 3769 and sizes.max() <= 3769 + 16
    parsed, item_start, status = oracle.decode_blocks(blocks, off, nthreads=3)
    assert (status == 0).all()
    assert int(item_start[-1]) == len(items)
    # same bytes as the single-block path
    for b in (0, 17, 39):
        payload = oracle.data_block_encode(it, int(starts[b]), int(starts[b + 1] - starts[b]))
        assert bytes(blocks[int(off[b]):int(off[b + 1])]) == oracle.block_write(payload)


def test_decode_rejects_corruption(oracle):
    items = [(b"k%03d" % i, b"v" * 10, i, 0) for i in range(40)]
    payload = oracle.data_block_encode(oracle.Items.from_list(items), restart_interval=4)
    blk = bytearray(oracle.block_write(payload))
    blocks = np.frombuffer(bytes(blk) * 1, np.uint8)
    off = np.array([0, len(blk)], np.uint64)
    assert oracle.decode_blocks(blocks, off)[2][0] == 0
    assert oracle.decode_blocks(blocks, off, expect_type=1)[2][0] == 7  # TYPE_MISMATCH
    # a structurally broken payload with a valid checksum -> PARSE
    bad = bytearray(payload)
    bad[0] = 9  # invalid value type at the first record
    blk2 = oracle.block_write(bytes(bad))
    assert oracle.decode_blocks(np.frombuffer(blk2, np.uint8), np.array([0, len(blk2)], np.uint64))[2][0] == 5


def test_oracle_asan():
    """The oracle under ASan/UBSan on the host: oracle/fuzz_driver.c
    runs seeded data_block fuzz properties (fuzz/data_block/src/main.rs:130-323:
    round trip, materialize == input, every point_read) plus re-sealed byte-flip
    mutations, truncated handles, random LZ4 streams and every XXH3 length class;
    any sanitizer report or failed property is a non-zero exit."""
    import subprocess
    from pathlib import Path
    oracle_dir = Path(__file__).resolve().parent.parent / "oracle"
    subprocess.run(["make", "-s", "-C", str(oracle_dir), "asan"], check=True)
    for seed in ("0x5EED", "0xC0FFEE", "7"):
        r = subprocess.run([str(oracle_dir / "fuzz_asan"), seed, "1500"], capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-4000:]
        assert "fuzz_driver ok" in r.stdout


def test_table_write_and_scanner(oracle):
    """pyoracle.table_write + scanner (Scanner, src/table/scanner.rs:24-92): the block
    index (full and two-level) lists exactly the data blocks, and the scanned items
    are the written items with global_seqno added."""
    from helpers import counter_items
    items = counter_items(52 * 30, seed=2)
    for two_level in (False, True):
        t = oracle.table_write(items, two_level=two_level, partition_size=600)
        tli = t["file"][t["tli_off"]:t["tli_off"] + t["tli_size"]]
        assert oracle.block_verify(tli)[0] == 0
        n, parsed = oracle.data_block_decode(tli[33:], index=True)
        handles = list(zip(parsed["handle_off"].tolist(), parsed["val_len"].tolist()))
        if two_level:
            assert n > 1 and handles[0][0] == t["index_off"]
            data_handles = []
            for o, sz in handles:
                m, p = oracle.data_block_decode(t["file"][o + 33:o + sz], index=True)
                data_handles += list(zip(p["handle_off"].tolist(), p["val_len"].tolist()))
            handles = data_handles
        assert [o for o, _ in handles] == t["block_off"][:-1].tolist()
        assert [o + s for o, s in handles] == t["block_off"][1:].tolist()
        blocks, err = oracle.scanner(t["file"], t["block_count"], 2 ** 64 - 1)
        assert err == 0 and len(blocks) == t["block_count"]
        seq = np.concatenate([b[2]["seqno"] for b in blocks])
        assert (seq == items.seqno - np.uint64(1)).all()  # + (2^64 - 1) wraps
        assert sum(len(b[2]["seqno"]) for b in blocks) == items.n
