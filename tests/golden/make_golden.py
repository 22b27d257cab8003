#!/usr/bin/env python3
"""Generate tests/golden/*.json — the committed golden vectors for the block codec.

This is a SECOND, independent restatement of the reference encoder, written in
pure Python on top of python-xxhash (libxxhash 0.8.2, the XXH3 that
xxhash-rust ^0.8.15 implements).  It shares no code with oracle/ (C) or the HIP
product; tests/test_oracle.py checks the C oracle against these vectors and
tests/test_gpu_parity.py checks the GPU path against them.

Reference files restated (fjall-rs/lsm-tree 3.1.9):
  src/table/block/encoder.rs:84-164, trailer.rs:78-173,
  binary_index/builder.rs:19-54, hash_index/builder.rs:18-124,
  src/table/data_block/mod.rs:195-264,523-549,
  src/table/index_block/mod.rs:110-127, block_handle.rs:134-156,
  src/table/block/mod.rs:45-84, header.rs:80-112.

The reference cannot run here (Rust, no cargo), so these vectors are pinned by
the reference's own KATs (src/hash.rs:17-31, hash_index/mod.rs:49-79) and the
hand-derived SURVEY.md Appendix B block, which are asserted below.

Run:  python tests/golden/make_golden.py   (rewrites the JSON files)
"""
from __future__ import annotations

import json
import random
import struct
from pathlib import Path

import numpy as np
import xxhash

OUT = Path(__file__).resolve().parent


def leb(v: int) -> bytes:
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def lcp(a: bytes, b: bytes) -> int:
    n = 0
    for x, y in zip(a, b):
        if x != y:
            break
        n += 1
    return n


def f32(x: float) -> float:
    return struct.unpack("<f", struct.pack("<f", x))[0]


def bucket_count(n: int, ratio: float) -> int:
    if not ratio > 0.0:
        return 0
    prod = f32(f32(float(n)) * f32(ratio))
    b = 0 if prod <= 0 else min(int(prod), 0xFFFFFFFF)
    return max(1, b)


def trailer(out: bytearray, ri: int, bin_idx, hash_bytes, n_items: int):
    out.append(0xFF)
    bin_off = len(out)
    step = 2 if bin_idx[-1] <= 0xFFFF else 4
    for x in bin_idx:
        out += struct.pack("<H" if step == 2 else "<I", x)
    hash_off = 0
    if hash_bytes is not None and len(hash_bytes) > 0 and len(bin_idx) <= 254:
        hash_off = len(out)
        out += bytes(hash_bytes)
    out += struct.pack("<BBIIII", ri, step, len(bin_idx), bin_off,
                       len(hash_bytes) if hash_off > 0 else 0, hash_off)
    out += struct.pack("<BBHBI", 1, 0, 0, 0, 0)
    out += struct.pack("<I", n_items)


def encode_data_block(items, ri: int, ratio: float) -> bytes:
    out = bytearray()
    bin_idx = []
    nb = bucket_count(len(items), ratio)
    hb = [254] * nb
    base = b""
    for i, (k, v, seq, vt) in enumerate(items):
        if i % ri == 0:
            bin_idx.append(len(out))
            out += bytes([vt]) + leb(seq) + leb(len(k)) + k
            base = k
        else:
            s = lcp(base, k)
            out += bytes([vt]) + leb(seq) + leb(s) + leb(len(k) - s) + k[s:]
        if vt not in (1, 2):
            out += leb(len(v)) + v
        ridx = len(bin_idx) - 1
        if nb > 0 and ridx < 254:
            pos = xxhash.xxh3_64_intdigest(k) % nb
            cur = hb[pos]
            if cur == 254:
                hb[pos] = ridx
            elif cur != 255 and cur != ridx:
                hb[pos] = 255
    trailer(out, ri, bin_idx, hb if nb else None, len(items))
    return bytes(out)


def encode_index_block(items) -> bytes:
    out = bytearray()
    bin_idx = []
    for (k, seq, off, size) in items:
        bin_idx.append(len(out))
        out += b"\x00" + leb(off) + leb(size) + leb(seq) + leb(len(k)) + k
    trailer(out, 1, bin_idx, None, len(items))
    return bytes(out)


def write_block(payload: bytes, block_type: int) -> bytes:
    h = xxhash.xxh3_128_intdigest(payload)
    hdr = b"LSM\x03" + bytes([block_type]) + h.to_bytes(16, "little") + struct.pack("<II", len(payload), len(payload))
    hdr += struct.pack("<I", xxhash.xxh3_128_intdigest(hdr) & 0xFFFFFFFF)
    return hdr + payload


def sorted_items(rng: random.Random, n: int, key_alphabet=b"abc", kmin=1, kmax=12, vmax=40,
                 mvcc=False, vtypes=(0, 1, 2, 4), big_seq=False):
    """Sorted, deduplicated (user_key asc, seqno desc) items like fuzz/data_block."""
    raw = {}
    for _ in range(n):
        k = bytes(rng.choice(key_alphabet) for _ in range(rng.randint(kmin, kmax)))
        seq = rng.getrandbits(63) if big_seq else rng.randint(0, 300)
        vt = rng.choice(vtypes)
        v = b"" if vt in (1, 2) else bytes(rng.getrandbits(8) for _ in range(rng.randint(0, vmax)))
        raw[(k, seq)] = (v, vt)
        if mvcc and rng.random() < 0.3:
            seq2 = seq + rng.randint(1, 5)
            vt2 = rng.choice(vtypes)
            v2 = b"" if vt2 in (1, 2) else b"mv" * rng.randint(0, 3)
            raw[(k, seq2)] = (v2, vt2)
    keys = sorted(raw.keys(), key=lambda ks: (ks[0], -ks[1]))
    return [(k, raw[(k, s)][0], s, raw[(k, s)][1]) for (k, s) in keys]


def h(b: bytes) -> str:
    return b.hex()


def main():
    # --- reference KATs that pin python-xxhash (src/hash.rs:17-31) -------------
    assert xxhash.xxh3_64_intdigest(bytes([0, 0, 0])) == 16_959_823_422_411_450_475
    assert xxhash.xxh3_64_intdigest(bytes([0, 0, 1])) == 8_004_557_073_989_523_290
    assert xxhash.xxh3_128_intdigest(bytes([0, 0, 0])) == 321_827_061_816_535_117_015_859_907_874_601_773_163
    assert xxhash.xxh3_128_intdigest(bytes([0, 0, 1])) == 154_036_699_985_066_753_773_347_827_765_470_844_762
    # --- hash_index/mod.rs:49-79: buckets of "a","b","c" mod 100 ----------------
    hb = [254] * 100
    for k, idx in ((b"a", 5), (b"b", 8), (b"c", 10)):
        hb[xxhash.xxh3_64_intdigest(k) % 100] = idx
    assert hb[11] == 10 and hb[15] == 8 and hb[19] == 5 and hb.count(254) == 97
    # --- SURVEY Appendix B ----------------------------------------------------
    appb = encode_data_block([(b"pla:earth:fact", b"eaaaaaaaaarth", 0, 0)], 16, 0.0)
    assert appb.hex() == ("00000e706c613a65617274683a666163740d65616161616161616161727468ff0000"
                          "1002010000002000000000000000000000000100000000000000000100000000"[:-2]), appb.hex()
    blk = write_block(appb, 0)
    assert blk[:33].hex() == "4c534d0300de4adbc6de9c817fcd96c0742a6fb32b4100000041000000e742de23"

    # --- xxh3 vectors: input_i = (31*i + 7) & 0xFF ------------------------------
    lens = list(range(0, 260)) + [383, 511, 512, 513, 1023, 1024, 1025, 1087, 2048, 3736, 4096, 4433,
                                  14920, 58276, 69186, 100003]
    kat = []
    for n in lens:
        b = bytes(((31 * i + 7) & 0xFF) for i in range(n))
        kat.append({"len": n, "xxh3_64": str(xxhash.xxh3_64_intdigest(b)),
                    "xxh3_128": str(xxhash.xxh3_128_intdigest(b))})
    (OUT / "xxh3_kat.json").write_text(json.dumps({"input": "(31*i+7)&0xFF", "vectors": kat}, indent=0))

    # --- block fixtures ---------------------------------------------------------
    rng = random.Random(0x5EED)
    cases = []

    def add_data(name, items, ri, ratio, block_type=0):
        payload = encode_data_block(items, ri, ratio)
        cases.append({
            "name": name, "kind": "data", "block_type": block_type, "restart_interval": ri,
            "hash_ratio": ratio,
            "items": [[h(k), h(v), str(s), t] for (k, v, s, t) in items],
            "block": h(write_block(payload, block_type)),
        })

    def add_index(name, items):
        payload = encode_index_block(items)
        cases.append({
            "name": name, "kind": "index", "block_type": 1, "restart_interval": 1, "hash_ratio": 0.0,
            "items": [[h(k), str(s), str(o), sz] for (k, s, o, sz) in items],
            "block": h(write_block(payload, 1)),
        })

    add_data("appendix_b", [(b"pla:earth:fact", b"eaaaaaaaaarth", 0, 0)], 16, 0.0)
    # data_block/mod.rs tests' shapes: restart intervals 1..16, hash ratio 0 / 1.0 / 1.33
    for ri in range(1, 17):
        for ratio in (0.0, 1.0, 1.33):
            items = sorted_items(rng, rng.randint(1, 60), mvcc=True)
            add_data(f"fuzzlike_ri{ri}_h{ratio}", items, ri, ratio)
    # big seqnos (10-byte LEB), long keys (2-byte key-len LEB), big values (3-byte LEB)
    big = sorted_items(rng, 20, kmin=130, kmax=300, vmax=0, big_seq=True, vtypes=(0,))
    big = [(k, bytes(rng.getrandbits(8) for _ in range(rng.choice([0, 127, 128, 16384, 20000]))), s, t)
           for (k, _, s, t) in big]
    big.append((b"\xff" * 5, b"x", 2 ** 64 - 1, 0))
    big.sort(key=lambda it: (it[0], -it[2]))
    add_data("max_varints", big, 4, 0.0)
    add_data("max_varints_ri1_hash", big, 1, 2.0)
    # tombstones only / weak tombstones / indirection
    add_data("tombstones", sorted_items(rng, 40, vtypes=(1, 2)), 16, 0.0)
    add_data("indirection", sorted_items(rng, 40, vtypes=(4,)), 8, 1.0)
    # u32 binary index: restart offsets > 65535
    many = [(b"key%06d" % i, bytes([i & 0xFF]) * 100, 7, 0) for i in range(900)]
    add_data("u32_binary_index", many, 16, 0.0)
    # hash index dropped when > 254 restarts (trailer.rs:100-111)
    add_data("hash_dropped_gt254", [(b"k%05d" % i, b"v", 1, 0) for i in range(300)], 1, 1.0)
    # hash index exactly at 254 restarts
    add_data("hash_at_254", [(b"k%05d" % i, b"v", 1, 0) for i in range(254)], 1, 1.0)
    # identical keys (shared == full key length, MVCC versions)
    add_data("mvcc_same_key", [(b"same", b"v%d" % s, s, 0) for s in range(30, 0, -1)], 4, 1.33)
    # meta block (DataBlock, RI 1, type Meta, writer/mod.rs:503-513)
    add_data("meta_block", [(b"#%s" % k, b"%d" % v, 0, 0) for k, v in
                            sorted([(b"data_count", 3), (b"item_count", 57), (b"key_count", 41)])], 1, 0.0, 3)
    # BASELINE config shapes (small counts)
    cnt = [(int(i).to_bytes(16, "big"), bytes(rng.getrandbits(8) for _ in range(64)), 63, 0) for i in range(52)]
    add_data("cfg1_4k_counter", cnt, 16, 0.0)
    pre = bytes(rng.getrandbits(8) for _ in range(32))
    ph = [(pre + int(i).to_bytes(8, "big"), bytes(rng.getrandbits(8) for _ in range(256)), 63, 0) for i in range(56)]
    add_data("cfg4_prefix_heavy_16k", ph, 16, 0.0)
    # index blocks
    for n in (1, 2, 17, 120):
        items = []
        off = 0
        for i in range(n):
            size = rng.randint(40, 70000)
            items.append((b"end%05d" % (i * 3), rng.getrandbits(63) if i % 3 == 0 else i, off, size))
            off += size
        add_index(f"index_{n}", items)

    (OUT / "blocks.json").write_text(json.dumps({"generator": "tests/golden/make_golden.py", "cases": cases}))
    print(f"wrote {len(cases)} block cases, {len(kat)} xxh3 vectors")


if __name__ == "__main__":
    main()
