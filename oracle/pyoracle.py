"""ctypes binding of oracle/liblsmoracle.so — TEST INFRASTRUCTURE ONLY.

Used by tests/ (as the checker), __graft_entry__.smoke() and bench.py's
cpu_baseline leg.  The product path (lsm-tree_amd/) never imports this.
See oracle/lsm_oracle.h for the reference citations.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB_PATH = HERE / "liblsmoracle.so"

u8p = C.POINTER(C.c_uint8)
u16p = C.POINTER(C.c_uint16)
u32p = C.POINTER(C.c_uint32)
u64p = C.POINTER(C.c_uint64)
i32p = C.POINTER(C.c_int32)


class OrcItems(C.Structure):
    _fields_ = [
        ("keys", u8p), ("key_off", u64p), ("vals", u8p), ("val_off", u64p),
        ("seqno", u64p), ("vtype", u8p), ("handle_off", u64p), ("handle_size", u32p),
        ("n_items", C.c_uint64),
    ]


class OrcParsed(C.Structure):
    _fields_ = [
        ("seqno", u64p), ("key_off", u32p), ("val_off", u32p), ("val_len", u32p),
        ("key_len", u16p), ("prefix_len", u16p), ("vtype", u8p), ("handle_off", u64p),
    ]


class OrcHeader(C.Structure):
    _fields_ = [("block_type", C.c_uint8), ("cksum_lo", C.c_uint64), ("cksum_hi", C.c_uint64),
                ("data_length", C.c_uint32), ("uncompressed_length", C.c_uint32)]


def build():
    import subprocess
    subprocess.run(["make", "-s", "-C", str(HERE)], check=True)


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            build()
        L = C.CDLL(str(LIB_PATH))
        L.orc_xxh3_64.restype = C.c_uint64
        L.orc_xxh3_64.argtypes = [C.c_void_p, C.c_size_t]
        L.orc_xxh3_128.restype = None
        L.orc_xxh3_128.argtypes = [C.c_void_p, C.c_size_t, u64p, u64p]
        L.orc_data_block_encode.restype = C.c_int64
        L.orc_data_block_encode.argtypes = [C.POINTER(OrcItems), C.c_uint64, C.c_uint64, C.c_uint8,
                                            C.c_float, C.c_void_p, C.c_size_t]
        L.orc_index_block_encode.restype = C.c_int64
        L.orc_index_block_encode.argtypes = [C.POINTER(OrcItems), C.c_uint64, C.c_uint64, C.c_void_p, C.c_size_t]
        L.orc_block_write.restype = C.c_int64
        L.orc_block_write.argtypes = [C.c_void_p, C.c_size_t, C.c_uint8, C.c_void_p, C.c_size_t]
        L.orc_header_decode.restype = C.c_int
        L.orc_header_decode.argtypes = [C.c_void_p, C.c_size_t, C.POINTER(OrcHeader)]
        L.orc_block_verify.restype = C.c_int
        L.orc_block_verify.argtypes = [C.c_void_p, C.c_size_t, C.POINTER(OrcHeader)]
        L.orc_data_block_decode.restype = C.c_int64
        L.orc_data_block_decode.argtypes = [C.c_void_p, C.c_size_t, C.POINTER(OrcParsed), C.c_uint64, C.c_uint64]
        L.orc_index_block_decode.restype = C.c_int64
        L.orc_index_block_decode.argtypes = [C.c_void_p, C.c_size_t, C.POINTER(OrcParsed), C.c_uint64, C.c_uint64]
        L.orc_data_block_point_read.restype = C.c_int64
        L.orc_data_block_point_read.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t, C.c_uint64]
        L.orc_cut_blocks.restype = C.c_uint64
        L.orc_cut_blocks.argtypes = [C.POINTER(OrcItems), C.c_uint32, C.c_void_p, C.c_uint64]
        L.orc_encode_blocks.restype = C.c_int
        L.orc_encode_blocks.argtypes = [C.POINTER(OrcItems), C.c_void_p, C.c_uint32, C.c_uint8, C.c_float,
                                        C.c_uint8, C.c_void_p, C.c_uint64, C.c_void_p, C.c_int]
        L.orc_decode_blocks.restype = C.c_int
        L.orc_decode_blocks.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_int, C.POINTER(OrcParsed),
                                        C.c_uint64, C.c_void_p, C.c_void_p, C.c_int]
        L.orc_decode_materialize_blocks.restype = C.c_uint64
        L.orc_decode_materialize_blocks.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_int, u64p]
        L.orc_bloom_calculate_m.restype = C.c_uint64
        L.orc_bloom_calculate_m.argtypes = [C.c_uint64, C.c_float]
        for f in (L.orc_bloom_shape_fpr, L.orc_bloom_shape_bpk):
            f.restype = C.c_int
            f.argtypes = [C.c_uint64, C.c_float, u64p, u64p]
        L.orc_bloom_build.restype = None
        L.orc_bloom_build.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64, C.c_uint64, C.c_void_p]
        L.orc_bloom_contains.restype = C.c_int
        L.orc_bloom_contains.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64]
        L.orc_data_block_seek.restype = C.c_int
        L.orc_data_block_seek.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t,
                                          C.c_uint32, u32p, u32p, u32p]
        L.orc_hash_index_build.restype = None
        L.orc_hash_index_build.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint32, C.c_void_p]
        L.orc_hash_index_get.restype = C.c_uint8
        L.orc_hash_index_get.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_size_t]
        L.orc_header_encode.restype = None
        L.orc_header_encode.argtypes = [C.c_uint8, C.c_uint64, C.c_uint64, C.c_uint32, C.c_uint32, C.c_void_p]
        L.orc_lz4_decompress.restype = C.c_int64
        L.orc_lz4_decompress.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64]
        _lib = L
    return _lib


def _ptr(a, t=C.c_void_p):
    if a is None:
        return None
    return C.cast(a.ctypes.data, t)


def xxh3_64(b: bytes) -> int:
    a = np.frombuffer(b, dtype=np.uint8) if len(b) else np.zeros(1, np.uint8)
    return lib().orc_xxh3_64(_ptr(a), len(b))


def xxh3_128(b: bytes) -> int:
    a = np.frombuffer(b, dtype=np.uint8) if len(b) else np.zeros(1, np.uint8)
    lo, hi = C.c_uint64(), C.c_uint64()
    lib().orc_xxh3_128(_ptr(a), len(b), C.byref(lo), C.byref(hi))
    return (hi.value << 64) | lo.value


BLOOM_HDR = 22


def bloom_calculate_m(n: int, fpr: float) -> int:
    """Builder::calculate_m (src/table/filter/standard_bloom/builder.rs:128-151)."""
    return lib().orc_bloom_calculate_m(n, fpr)


def bloom_shape(n: int, bpk: float | None = None, fpr: float | None = None):
    """BloomConstructionPolicy::init (src/table/filter/mod.rs:25-34) -> (m, k)."""
    m, k = C.c_uint64(), C.c_uint64()
    f = lib().orc_bloom_shape_bpk if bpk is not None else lib().orc_bloom_shape_fpr
    rc = f(n, bpk if bpk is not None else fpr, C.byref(m), C.byref(k))
    if rc:
        raise ValueError("bloom shape: n must be > 0 (and bpk > 0)")
    return m.value, k.value


def bloom_build(hashes: np.ndarray, m: int, k: int) -> bytes:
    """set_with_hash for every hash, then Builder::build (builder.rs:33-53,154-170)."""
    h = np.ascontiguousarray(hashes, dtype=np.uint64)
    out = np.zeros(BLOOM_HDR + m // 8, np.uint8)
    lib().orc_bloom_build(_ptr(h) if len(h) else None, len(h), m, k, _ptr(out))
    return out.tobytes()


def bloom_contains(filt: bytes, h: int) -> int:
    """StandardBloomFilterReader::contains_hash (standard_bloom/mod.rs:100-120)."""
    a = np.frombuffer(filt, np.uint8)
    return lib().orc_bloom_contains(_ptr(a), len(filt), h)


def lz4_decompress(src: bytes, cap: int):
    """LZ4 block decode (lz4_flex::decompress_into, src/table/block/mod.rs:104-118) -> bytes or None."""
    a = np.frombuffer(src, np.uint8) if len(src) else np.zeros(1, np.uint8)
    out = np.zeros(max(cap, 1), np.uint8)
    n = lib().orc_lz4_decompress(_ptr(a), len(src), _ptr(out), cap)
    return None if n < 0 else out[:n].tobytes()


def block_header(block_type: int, payload: bytes, uncompressed_length: int) -> bytes:
    """Header::encode_into (src/table/block/header.rs:80-112) for a payload as stored
    (compressed or not): checksum = xxh3_128(stored payload)."""
    ck = xxh3_128(payload)
    h = b"LSM\x03" + bytes([block_type]) + ck.to_bytes(16, "little") + len(payload).to_bytes(4, "little") + \
        uncompressed_length.to_bytes(4, "little")
    return h + (xxh3_128(h) & 0xFFFFFFFF).to_bytes(4, "little")


class Items:
    """Host SoA item batch (same layout as include/lsmgpu.h lsm_items)."""

    def __init__(self, keys, key_off, vals, val_off, seqno, vtype, handle_off=None, handle_size=None):
        self.keys = np.ascontiguousarray(keys, dtype=np.uint8)
        self.key_off = np.ascontiguousarray(key_off, dtype=np.uint64)
        self.vals = np.ascontiguousarray(vals, dtype=np.uint8)
        self.val_off = np.ascontiguousarray(val_off, dtype=np.uint64)
        self.seqno = np.ascontiguousarray(seqno, dtype=np.uint64)
        self.vtype = np.ascontiguousarray(vtype, dtype=np.uint8)
        n = len(self.seqno)
        self.handle_off = np.ascontiguousarray(handle_off if handle_off is not None else np.zeros(n), dtype=np.uint64)
        self.handle_size = np.ascontiguousarray(handle_size if handle_size is not None else np.zeros(n), dtype=np.uint32)
        self.n = n
        if len(self.keys) == 0:
            self.keys = np.zeros(1, np.uint8)
        if len(self.vals) == 0:
            self.vals = np.zeros(1, np.uint8)

    @classmethod
    def from_list(cls, items):
        """items: list of (key bytes, value bytes, seqno, vtype) or index tuples
        (key, seqno, handle_offset, handle_size) when len==4 and value is int."""
        keys = b"".join(k for k, *_ in items)
        kl = np.array([len(k) for k, *_ in items], dtype=np.uint64)
        key_off = np.concatenate([[0], np.cumsum(kl)]).astype(np.uint64)
        vals = b"".join(v for _, v, _, _ in items)
        vl = np.array([len(v) for _, v, _, _ in items], dtype=np.uint64)
        val_off = np.concatenate([[0], np.cumsum(vl)]).astype(np.uint64)
        seq = np.array([s for _, _, s, _ in items], dtype=np.uint64)
        vt = np.array([t for _, _, _, t in items], dtype=np.uint8)
        return cls(np.frombuffer(keys, np.uint8), key_off, np.frombuffer(vals, np.uint8), val_off, seq, vt)

    def struct(self) -> OrcItems:
        s = OrcItems()
        s.keys = _ptr(self.keys, u8p); s.key_off = _ptr(self.key_off, u64p)
        s.vals = _ptr(self.vals, u8p); s.val_off = _ptr(self.val_off, u64p)
        s.seqno = _ptr(self.seqno, u64p); s.vtype = _ptr(self.vtype, u8p)
        s.handle_off = _ptr(self.handle_off, u64p); s.handle_size = _ptr(self.handle_size, u32p)
        s.n_items = self.n
        return s


def data_block_encode(items: Items, first=0, count=None, restart_interval=16, hash_ratio=0.0) -> bytes:
    count = items.n - first if count is None else count
    cap = 64 + 3 * (len(items.keys) + len(items.vals)) + 64 * count + 2 * 1024 * 1024
    out = np.zeros(cap, np.uint8)
    s = items.struct()
    n = lib().orc_data_block_encode(C.byref(s), first, count, restart_interval, hash_ratio, _ptr(out), cap)
    if n < 0:
        raise ValueError(f"encode failed status {-n}")
    return out[:n].tobytes()


def index_block_encode(items: Items, first=0, count=None) -> bytes:
    count = items.n - first if count is None else count
    cap = 64 + 3 * len(items.keys) + 64 * count + 4096
    out = np.zeros(cap, np.uint8)
    s = items.struct()
    n = lib().orc_index_block_encode(C.byref(s), first, count, _ptr(out), cap)
    if n < 0:
        raise ValueError(f"encode failed status {-n}")
    return out[:n].tobytes()


def block_write(payload: bytes, block_type=0) -> bytes:
    cap = len(payload) + 33
    out = np.zeros(cap, np.uint8)
    src = np.frombuffer(payload, np.uint8) if payload else np.zeros(1, np.uint8)
    n = lib().orc_block_write(_ptr(src), len(payload), block_type, _ptr(out), cap)
    if n < 0:
        raise ValueError(f"write failed {-n}")
    return out[:n].tobytes()


def header_decode(buf: bytes):
    h = OrcHeader()
    a = np.frombuffer(buf, np.uint8) if buf else np.zeros(1, np.uint8)
    st = lib().orc_header_decode(_ptr(a), len(buf), C.byref(h))
    return st, h


def block_verify(buf: bytes):
    h = OrcHeader()
    a = np.frombuffer(buf, np.uint8) if buf else np.zeros(1, np.uint8)
    st = lib().orc_block_verify(_ptr(a), len(buf), C.byref(h))
    return st, h


class Parsed:
    FIELDS = (("seqno", np.uint64), ("key_off", np.uint32), ("val_off", np.uint32), ("val_len", np.uint32),
              ("key_len", np.uint16), ("prefix_len", np.uint16), ("vtype", np.uint8), ("handle_off", np.uint64))

    def __init__(self, n):
        for name, dt in self.FIELDS:
            setattr(self, name, np.zeros(max(n, 1), dt))
        self.n = n

    def struct(self) -> OrcParsed:
        s = OrcParsed()
        s.seqno = _ptr(self.seqno, u64p); s.key_off = _ptr(self.key_off, u32p)
        s.val_off = _ptr(self.val_off, u32p); s.val_len = _ptr(self.val_len, u32p)
        s.key_len = _ptr(self.key_len, u16p); s.prefix_len = _ptr(self.prefix_len, u16p)
        s.vtype = _ptr(self.vtype, u8p); s.handle_off = _ptr(self.handle_off, u64p)
        return s

    def trimmed(self, n):
        return {name: getattr(self, name)[:n].copy() for name, _ in self.FIELDS}


def data_block_decode(payload: bytes, cap=None, index=False):
    a = np.frombuffer(payload, np.uint8)
    cap = cap if cap is not None else max(1, len(payload))
    p = Parsed(cap)
    s = p.struct()
    fn = lib().orc_index_block_decode if index else lib().orc_data_block_decode
    n = fn(_ptr(a), len(payload), C.byref(s), 0, cap)
    if n < 0:
        return int(n), None
    return int(n), p.trimmed(n)


def materialize(payload: bytes, parsed: dict, restart_interval: int):
    """DataBlockParsedItem::materialize (data_block/mod.rs:296-315) in Python."""
    out = []
    n = len(parsed["seqno"])
    for i in range(n):
        h = (i // restart_interval) * restart_interval
        ko, kl, pl = int(parsed["key_off"][i]), int(parsed["key_len"][i]), int(parsed["prefix_len"][i])
        hk = int(parsed["key_off"][h])
        key = payload[hk:hk + pl] + payload[ko:ko + kl]
        vt = int(parsed["vtype"][i])
        vo, vl = int(parsed["val_off"][i]), int(parsed["val_len"][i])
        val = b"" if vt in (1, 2) else payload[vo:vo + vl]
        out.append((key, val, int(parsed["seqno"][i]), vt))
    return out


def point_read(payload: bytes, needle: bytes, snapshot: int) -> int:
    a = np.frombuffer(payload, np.uint8)
    nd = np.frombuffer(needle, np.uint8) if needle else np.zeros(1, np.uint8)
    return int(lib().orc_data_block_point_read(_ptr(a), len(payload), _ptr(nd), len(needle), snapshot))


SEEK_LO, SEEK_HI, SEEK_LO_EXCL, SEEK_HI_EXCL = 1, 2, 4, 8


def _arr(b: bytes):
    return np.frombuffer(b, np.uint8) if b else np.zeros(1, np.uint8)


def seek(payload: bytes, lo: bytes | None = None, hi: bytes | None = None, lo_excl=False, hi_excl=False):
    """Iter::seek / seek_upper (+ exclusive forms) (data_block/iter.rs:37-176) ->
    (first, end, lo_found, hi_found) or None for a malformed block."""
    flags = (SEEK_LO if lo is not None else 0) | (SEEK_HI if hi is not None else 0) | \
            (SEEK_LO_EXCL if lo_excl else 0) | (SEEK_HI_EXCL if hi_excl else 0)
    a, la, b, lb = _arr(lo or b""), len(lo or b""), _arr(hi or b""), len(hi or b"")
    first, end, found = C.c_uint32(), C.c_uint32(), C.c_uint32()
    rc = lib().orc_data_block_seek(_ptr(_arr(payload)), len(payload), _ptr(a), la, _ptr(b), lb, flags,
                                   C.byref(first), C.byref(end), C.byref(found))
    if rc:
        return None
    return first.value, end.value, bool(found.value & 1), bool(found.value & 2)


def hash_index_build(keys: list, idx: list, buckets: int) -> bytes:
    """hash_index::Builder::with_bucket_count(buckets) + set(key, idx)... + into_inner."""
    kb = b"".join(keys)
    ko = np.concatenate([[0], np.cumsum([len(k) for k in keys])]).astype(np.uint64)
    ix = np.array(idx, np.uint8) if idx else np.zeros(1, np.uint8)
    out = np.zeros(max(buckets, 1), np.uint8)
    lib().orc_hash_index_build(_ptr(_arr(kb)), _ptr(ko), _ptr(ix), len(keys), buckets, _ptr(out))
    return out[:buckets].tobytes()


def hash_index_get(bytes_: bytes, key: bytes) -> int:
    return lib().orc_hash_index_get(_ptr(_arr(bytes_)), len(bytes_), _ptr(_arr(key)), len(key))


def header_encode(block_type: int, checksum: int, data_length: int, uncompressed_length: int) -> bytes:
    out = np.zeros(33, np.uint8)
    lib().orc_header_encode(block_type, checksum & (2 ** 64 - 1), checksum >> 64, data_length, uncompressed_length,
                            _ptr(out))
    return out.tobytes()


def cut_blocks(items: Items, block_size: int) -> np.ndarray:
    starts = np.zeros(items.n + 2, np.uint32)
    s = items.struct()
    nb = lib().orc_cut_blocks(C.byref(s), block_size, _ptr(starts), items.n + 1)
    return starts[:nb + 1].copy()


def encode_blocks(items: Items, starts: np.ndarray, restart_interval=16, hash_ratio=0.0, block_type=0,
                  nthreads=None):
    nthreads = nthreads or os.cpu_count() or 1
    nb = len(starts) - 1
    starts = np.ascontiguousarray(starts, dtype=np.uint32)
    cap = 64 * nb + 3 * (len(items.keys) + len(items.vals)) + 64 * items.n + 4096
    out = np.zeros(cap, np.uint8)
    off = np.zeros(nb + 1, np.uint64)
    s = items.struct()
    rc = lib().orc_encode_blocks(C.byref(s), _ptr(starts), nb, restart_interval, hash_ratio, block_type,
                                 _ptr(out), cap, _ptr(off), nthreads)
    if rc != 0:
        raise ValueError(f"orc_encode_blocks failed status {-rc}")
    return out[:int(off[-1])], off


def decode_blocks(blocks: np.ndarray, block_off: np.ndarray, expect_type=-1, nthreads=None, item_cap=None):
    nthreads = nthreads or os.cpu_count() or 1
    nb = len(block_off) - 1
    blocks = np.ascontiguousarray(blocks, dtype=np.uint8)
    block_off = np.ascontiguousarray(block_off, dtype=np.uint64)
    if item_cap is None:
        item_cap = len(blocks) // 3 + 1
    p = Parsed(item_cap)
    item_start = np.zeros(nb + 1, np.uint32)
    status = np.zeros(max(nb, 1), np.int32)
    s = p.struct()
    lib().orc_decode_blocks(_ptr(blocks), _ptr(block_off), nb, expect_type, C.byref(s), item_cap,
                            _ptr(item_start), _ptr(status), nthreads)
    n = int(item_start[-1])
    return p.trimmed(n), item_start, status[:nb]


def decode_materialize_blocks(blocks: np.ndarray, block_off: np.ndarray, nthreads=1):
    fold = C.c_uint64()
    n = lib().orc_decode_materialize_blocks(_ptr(np.ascontiguousarray(blocks)), _ptr(np.ascontiguousarray(block_off, dtype=np.uint64)),
                                            len(block_off) - 1, nthreads, C.byref(fold))
    return int(n), fold.value


# ---- table file image + Scanner ------------------------------------

def table_write(items: Items, block_size=4096, restart_interval=16, hash_ratio=0.0, two_level=False,
                partition_size=4096):
    """Data and block-index regions of a table file (test fixture builder; the sfa TOC,
    meta, filter and trailer sections are not written — the caller gets the TLI handle
    the TOC would hold, regions.rs:55-76).
      Writer::write / spill_block (src/table/writer/mod.rs:243-343): items cut by
        cut_blocks, data blocks back to back from offset 0, each registered as
        KeyedBlockHandle(last key, last seqno, (file_pos, 33 + data_length));
      FullIndexWriter::finish (writer/index/full.rs:55-69): one TLI index block of all
        data-block handles;
      PartitionedIndexWriter (writer/index/partitioned.rs:54-125,158-235): handles are
        buffered and a partition index block is cut once the buffered size reaches
        partition_size (buffered size per handle = end_key length + 48, standing in for
        size_of::<KeyedBlockHandle>(), which is not pinned; the scan does not depend on
        where partitions are cut), partitions are concatenated as the "index" region
        after the data, and the TLI lists the partitions with handles shifted to file
        offsets (partitioned.rs:136-140).
    Returns dict(file bytes, tli_off, tli_size, index_off, data_len, block_count,
    block_off (data blocks), starts)."""
    starts = cut_blocks(items, block_size)
    data, off = encode_blocks(items, starts, restart_interval=restart_interval, hash_ratio=hash_ratio)
    nb = len(starts) - 1
    last = starts[1:] - 1
    ko = items.key_off

    def end_key(i):
        return items.keys[int(ko[i]):int(ko[i + 1])].tobytes()

    handles = [(end_key(int(j)), int(items.seqno[int(j)]), int(off[b]), int(off[b + 1] - off[b]))
               for b, j in enumerate(last)]

    def index_block(entries):
        it = Items(np.frombuffer(b"".join(k for k, *_ in entries), np.uint8),
                   np.concatenate([[0], np.cumsum([len(k) for k, *_ in entries])]).astype(np.uint64),
                   np.zeros(0, np.uint8), np.zeros(len(entries) + 1, np.uint64),
                   [s for _, s, _, _ in entries], np.zeros(len(entries), np.uint8),
                   [o for _, _, o, _ in entries], [z for _, _, _, z in entries])
        return block_write(index_block_encode(it), block_type=1)

    body = data.tobytes()
    index_off = len(body)
    if two_level:
        parts, buf, size, rel = [], [], 0, 0
        region = b""
        for h in handles:
            buf.append(h)
            size += len(h[0]) + 48
            if size >= partition_size:
                blk = index_block(buf)
                parts.append((buf[-1][0], buf[-1][1], index_off + rel, len(blk)))
                region += blk
                rel += len(blk)
                buf, size = [], 0
        if buf:
            blk = index_block(buf)
            parts.append((buf[-1][0], buf[-1][1], index_off + rel, len(blk)))
            region += blk
        body += region
        tli = index_block(parts)
    else:
        tli = index_block(handles)
    tli_off = len(body)
    body += tli
    return {"file": body, "tli_off": tli_off, "tli_size": len(tli), "index_off": index_off,
            "data_len": index_off, "block_count": nb, "block_off": off, "starts": starts}


def scanner(file: bytes, block_count: int, global_seqno: int = 0):
    """Scanner::new / next (src/table/scanner.rs:24-92): block_count blocks read back to
    back from offset 0 with Block::from_reader (header, then data_length payload bytes,
    xxh3 verify), each must be a Data block (fetch_next_block :54-72), every item's seqno
    += global_seqno (:84, wrapping as in release builds).  Iteration stops at the first
    error.  Returns (blocks, status): blocks = list of (offset, size, parsed dict) read
    before the error; status = 0 or the failing block's status."""
    pos, out = 0, []
    buf = np.frombuffer(file, np.uint8)
    for _ in range(block_count):
        st, h = header_decode(file[pos:pos + 33])
        if st:
            return out, st
        size = 33 + int(h.data_length)
        if pos + size > len(file):
            return out, 8  # Error::Io (UnexpectedEof): TRUNCATED
        parsed, item_start, status = decode_blocks(buf[pos:pos + size], np.array([0, size], np.uint64),
                                                   expect_type=0, nthreads=1)
        if status[0]:
            return out, int(status[0])
        parsed["seqno"] = (parsed["seqno"] + np.uint64(global_seqno & (2 ** 64 - 1))).astype(np.uint64)
        out.append((pos, size, parsed))
        pos += size
    return out, 0
