"""ctypes binding of lsm-tree_amd/liblsmgpu.so (include/lsmgpu.h) for tests and bench.

Device memory comes from torch CUDA tensors (plumbing only).  Every call goes
through the C ABI; there is no CPU fallback: importing this module on a box
without the built library raises, and calls without a GPU fail loudly.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

HERE = Path(__file__).resolve().parent
# LSMGPU_LIB: diagnostic override (tuning sweeps load variant builds of the same library)
LIB_PATH = Path(os.environ.get("LSMGPU_LIB", HERE / "liblsmgpu.so"))

LSM_HEADER_LEN = 33
LSM_TRAILER_LEN = 31
LSM_INPUT_PADDING = 64

STATUS = {0: "OK", 1: "BAD_MAGIC", 2: "BAD_TYPE", 3: "HDR_CKSUM", 4: "CKSUM", 5: "PARSE", 6: "OVERFLOW",
          7: "TYPE_MISMATCH", 8: "TRUNCATED", 9: "UNSUPPORTED", 10: "BAD_ARG", 11: "HIP_ERROR",
          12: "DECOMPRESS", 13: "INCOMPLETE"}
BLOCK_DATA, BLOCK_INDEX, BLOCK_FILTER, BLOCK_META = 0, 1, 2, 3


class LsmItems(C.Structure):
    _fields_ = [("keys", C.c_void_p), ("key_off", C.c_void_p), ("vals", C.c_void_p), ("val_off", C.c_void_p),
                ("seqno", C.c_void_p), ("vtype", C.c_void_p), ("handle_off", C.c_void_p),
                ("handle_size", C.c_void_p), ("n_items", C.c_uint64)]


class LsmItems32(C.Structure):  # lsm_items32: u32 key / value offsets (lsm_encode_blocks32)
    _fields_ = [("keys", C.c_void_p), ("key_off", C.c_void_p), ("vals", C.c_void_p), ("val_off", C.c_void_p),
                ("seqno", C.c_void_p), ("vtype", C.c_void_p), ("handle_off", C.c_void_p),
                ("handle_size", C.c_void_p), ("n_items", C.c_uint64)]


class LsmParsed(C.Structure):
    _fields_ = [("seqno", C.c_void_p), ("key_off", C.c_void_p), ("val_off", C.c_void_p), ("val_len", C.c_void_p),
                ("key_len", C.c_void_p), ("prefix_len", C.c_void_p), ("vtype", C.c_void_p),
                ("handle_off", C.c_void_p)]


class LsmParsed16(C.Structure):
    _fields_ = [("seqno", C.c_void_p), ("key_off", C.c_void_p), ("val_off", C.c_void_p), ("val_len", C.c_void_p),
                ("key_len", C.c_void_p), ("prefix_len", C.c_void_p), ("vtype", C.c_void_p)]


class LsmBlockParams(C.Structure):
    _fields_ = [("restart_interval", C.c_uint8), ("block_type", C.c_uint8), ("compression", C.c_uint8),
                ("reserved", C.c_uint8), ("hash_ratio", C.c_float), ("flags", C.c_uint32)]


class LsmPointResult(C.Structure):
    _fields_ = [("item", C.c_void_p), ("seqno", C.c_void_p), ("val_off", C.c_void_p), ("val_len", C.c_void_p),
                ("vtype", C.c_void_p)]


class LsmDecodeTuning(C.Structure):
    _fields_ = [("blocks_per_wave", C.c_uint32), ("stage_bytes", C.c_uint32), ("tile_items", C.c_uint32),
                ("flags", C.c_uint32)]


class LsmTableScan(C.Structure):
    _fields_ = [("tli_off", C.c_uint64), ("tli_size", C.c_uint32), ("two_level", C.c_uint32),
                ("global_seqno", C.c_uint64), ("block_count", C.c_uint64)]


ABI_VERSION = 7
DECODE_ITEM_START_VALID = 1
# lsm_decode_tuning.flags / lsm_block_params.flags: take the workspace pool (explicit opt-in)
DECODE_HUGE_POOL = 4
ENCODE_HUGE_POOL = 1
ENCODE_RUN_PLAN = 2
# Mean block size (bytes) from which the wrappers hand the workspace pool for
# blocks spread over the GPU (blocks > 72 KiB decode, > 96 KiB images encode).
HUGE_AUTO_MEAN = 32 << 10
DECODE_PAYLOAD_VERIFIED = 2


class LsmError(RuntimeError):
    pass


def build():
    import subprocess
    subprocess.run(["make", "-s", "-C", str(HERE), "-j8"], check=True)


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            raise LsmError(f"{LIB_PATH} not built: run `make -C {HERE}` (or __graft_entry__.build())")
        L = C.CDLL(str(LIB_PATH))
        L.lsm_abi_version.restype = C.c_int
        L.lsm_status_name.restype = C.c_char_p
        L.lsm_status_name.argtypes = [C.c_int]
        L.lsm_last_error.restype = C.c_char_p
        L.lsm_device_count.restype = C.c_int
        L.lsm_set_device.restype = C.c_int
        L.lsm_set_device.argtypes = [C.c_int]
        L.lsm_decode_workspace_size.restype = C.c_size_t
        L.lsm_decode_workspace_size.argtypes = [C.c_uint32]
        L.lsm_decode_workspace_size_ex.restype = C.c_size_t
        L.lsm_decode_workspace_size_ex.argtypes = [C.c_uint32, C.c_uint64]
        L.lsm_decode_blocks.restype = C.c_int
        L.lsm_decode_blocks.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_int32, C.POINTER(LsmParsed),
                                        C.c_uint64, C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p]
        L.lsm_decode_blocks_tuned.restype = C.c_int
        L.lsm_decode_blocks_tuned.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_int32, C.POINTER(LsmParsed),
                                              C.c_uint64, C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t,
                                              C.POINTER(LsmDecodeTuning), C.c_void_p]
        L.lsm_decode_blocks16.restype = C.c_int
        L.lsm_decode_blocks16.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_int32, C.POINTER(LsmParsed16),
                                          C.c_uint64, C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t,
                                          C.POINTER(LsmDecodeTuning), C.c_void_p]
        L.lsm_encode_bound.restype = C.c_uint64
        L.lsm_encode_bound.argtypes = [C.c_uint64, C.c_uint32, C.c_uint64, C.c_uint64, C.POINTER(LsmBlockParams)]
        L.lsm_encode_workspace_size.restype = C.c_size_t
        L.lsm_encode_workspace_size.argtypes = [C.c_uint64, C.c_uint32]
        L.lsm_encode_workspace_size_ex.restype = C.c_size_t
        L.lsm_encode_workspace_size_ex.argtypes = [C.c_uint64, C.c_uint32, C.c_uint64]
        L.lsm_encode_blocks.restype = C.c_int
        L.lsm_encode_blocks.argtypes = [C.POINTER(LsmItems), C.c_void_p, C.c_uint32, C.POINTER(LsmBlockParams),
                                        C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t,
                                        C.c_void_p]
        if hasattr(L, "lsm_encode_blocks32"):  # (variant builds of earlier trees lack it: A/B scripts)
            L.lsm_encode_blocks32.restype = C.c_int
            L.lsm_encode_blocks32.argtypes = [C.POINTER(LsmItems32), C.c_void_p, C.c_uint32,
                                              C.POINTER(LsmBlockParams), C.c_void_p, C.c_uint64, C.c_void_p,
                                              C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p]
        L.lsm_cut_blocks.restype = C.c_uint64
        L.lsm_cut_blocks.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint32, C.c_void_p, C.c_uint64]
        L.lsm_xxh3_128_batch.restype = C.c_int
        L.lsm_xxh3_128_batch.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p]
        L.lsm_xxh3_128_file_workspace_size.restype = C.c_size_t
        L.lsm_xxh3_128_file_workspace_size.argtypes = [C.c_uint64]
        L.lsm_xxh3_128_file.restype = C.c_int
        L.lsm_xxh3_128_file.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p]
        L.lsm_xxh3_128_stream_state_size.restype = C.c_size_t
        L.lsm_xxh3_128_stream_state_size.argtypes = []
        L.lsm_xxh3_128_stream_workspace_size.restype = C.c_size_t
        L.lsm_xxh3_128_stream_workspace_size.argtypes = [C.c_uint64]
        L.lsm_xxh3_128_stream_init.restype = C.c_int
        L.lsm_xxh3_128_stream_init.argtypes = [C.c_void_p, C.c_void_p]
        L.lsm_xxh3_128_stream_update.restype = C.c_int
        L.lsm_xxh3_128_stream_update.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p, C.c_size_t,
                                                 C.c_void_p]
        L.lsm_xxh3_128_stream_digest.restype = C.c_int
        L.lsm_xxh3_128_stream_digest.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
        L.lsm_xxh3_128_stream_init_batch.restype = C.c_int
        L.lsm_xxh3_128_stream_init_batch.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p]
        L.lsm_xxh3_128_stream_batch_workspace_size.restype = C.c_size_t
        L.lsm_xxh3_128_stream_batch_workspace_size.argtypes = [C.c_uint32, C.c_uint64]
        L.lsm_xxh3_128_stream_update_batch.restype = C.c_int
        L.lsm_xxh3_128_stream_update_batch.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_uint64,
                                                       C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p]
        L.lsm_xxh3_128_stream_digest_batch.restype = C.c_int
        L.lsm_xxh3_128_stream_digest_batch.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p]
        L.lsm_point_read_blocks.restype = C.c_int
        L.lsm_point_read_blocks.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p,
                                            C.c_void_p, C.c_uint32, C.POINTER(LsmPointResult), C.c_void_p,
                                            C.c_void_p]
        L.lsm_seek_blocks.restype = C.c_int
        L.lsm_seek_blocks.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p,
                                      C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p,
                                      C.c_void_p, C.c_void_p, C.c_void_p]
        L.lsm_bloom_calculate_m.restype = C.c_uint64
        L.lsm_bloom_calculate_m.argtypes = [C.c_uint64, C.c_float]
        L.lsm_bloom_shape.restype = C.c_int
        L.lsm_bloom_shape.argtypes = [C.c_uint64, C.c_int, C.c_float, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
        L.lsm_bloom_filter_size.restype = C.c_uint64
        L.lsm_bloom_filter_size.argtypes = [C.c_uint64]
        L.lsm_hash64_keys.restype = C.c_int
        L.lsm_hash64_keys.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p]
        L.lsm_bloom_build.restype = C.c_int
        L.lsm_bloom_build.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64, C.c_uint64, C.c_void_p, C.c_uint64,
                                      C.c_void_p]
        L.lsm_bloom_contains.restype = C.c_int
        L.lsm_bloom_contains.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p]
        L.lsm_lz4_workspace_size.restype = C.c_size_t
        L.lsm_lz4_workspace_size.argtypes = [C.c_uint32]
        L.lsm_lz4_decompress_blocks.restype = C.c_int
        L.lsm_lz4_decompress_blocks.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p,
                                                C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p]
        L.lsm_lz4_plan_workspace_size.restype = C.c_size_t
        L.lsm_lz4_plan_workspace_size.argtypes = [C.c_uint32]
        L.lsm_lz4_plan_output.restype = C.c_int
        L.lsm_lz4_plan_output.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint64, C.c_void_p, C.c_void_p,
                                          C.c_size_t, C.c_void_p]
        for fn in (L.lsm_lz4_plan_framed,):
            fn.restype = C.c_int
            fn.argtypes = L.lsm_lz4_plan_output.argtypes
        L.lsm_lz4_decompress_framed.restype = C.c_int
        L.lsm_lz4_decompress_framed.argtypes = L.lsm_lz4_decompress_blocks.argtypes
        L.lsm_scan_workspace_size.restype = C.c_size_t
        L.lsm_scan_workspace_size.argtypes = [C.c_uint32]
        L.lsm_scan_table_async.restype = C.c_int
        L.lsm_scan_table_async.argtypes = [C.c_void_p, C.c_uint64, C.POINTER(LsmTableScan), C.c_void_p, C.c_uint32,
                                           C.c_uint32, C.c_uint32, C.POINTER(LsmParsed), C.c_uint64, C.c_void_p, C.c_void_p,
                                           C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p]
        L.lsm_scan_table.restype = C.c_int
        L.lsm_scan_table.argtypes = [C.c_void_p, C.c_uint64, C.POINTER(LsmTableScan), C.c_void_p, C.c_uint32,
                                     C.POINTER(LsmParsed), C.c_uint64, C.c_void_p, C.c_void_p,
                                     C.POINTER(C.c_uint32), C.POINTER(C.c_int32), C.c_void_p, C.c_size_t, C.c_void_p]
        L.lsm_materialize_workspace_size.restype = C.c_size_t
        L.lsm_materialize_workspace_size.argtypes = [C.c_uint64]
        L.lsm_materialize_plan.restype = C.c_int
        L.lsm_materialize_plan.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p,
                                           C.POINTER(LsmParsed), C.c_uint64, C.c_void_p, C.c_void_p, C.c_size_t,
                                           C.c_void_p]
        L.lsm_materialize_keys_capped.restype = C.c_int
        L.lsm_materialize_keys_capped.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p,
                                                  C.POINTER(LsmParsed), C.c_uint64, C.c_void_p, C.c_void_p,
                                                  C.c_uint64, C.c_void_p, C.c_void_p]
        L.lsm_lz4_plan_capped.restype = C.c_int
        L.lsm_lz4_plan_capped.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint64, C.c_int, C.c_uint64,
                                          C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p]
        L.lsm_materialize_keys.restype = C.c_int
        L.lsm_materialize_keys.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p,
                                           C.POINTER(LsmParsed), C.c_uint64, C.c_void_p, C.c_void_p, C.c_void_p]
        _lib = L
    return _lib


EXPORTED_SYMBOLS = ["lsm_abi_version", "lsm_status_name", "lsm_last_error", "lsm_device_count", "lsm_set_device",
                    "lsm_decode_workspace_size", "lsm_decode_workspace_size_ex", "lsm_decode_blocks", "lsm_decode_blocks_tuned", "lsm_decode_blocks16",
                    "lsm_encode_bound",
                    "lsm_encode_workspace_size", "lsm_encode_workspace_size_ex", "lsm_encode_blocks", "lsm_encode_blocks32",
                    "lsm_cut_blocks", "lsm_xxh3_128_batch",
                    "lsm_point_read_blocks", "lsm_xxh3_128_file_workspace_size", "lsm_xxh3_128_file",
                    "lsm_bloom_calculate_m", "lsm_bloom_shape", "lsm_bloom_filter_size", "lsm_hash64_keys",
                    "lsm_bloom_build", "lsm_bloom_contains", "lsm_lz4_workspace_size", "lsm_lz4_decompress_blocks",
                    "lsm_lz4_plan_workspace_size", "lsm_lz4_plan_output", "lsm_seek_blocks", "lsm_lz4_plan_framed",
                    "lsm_lz4_decompress_framed", "lsm_scan_workspace_size", "lsm_scan_table", "lsm_scan_table_async",
                    "lsm_materialize_workspace_size", "lsm_materialize_plan", "lsm_materialize_keys",
                    "lsm_materialize_keys_capped", "lsm_lz4_plan_capped",
                    "lsm_xxh3_128_stream_state_size", "lsm_xxh3_128_stream_workspace_size",
                    "lsm_xxh3_128_stream_init", "lsm_xxh3_128_stream_update", "lsm_xxh3_128_stream_digest",
                    "lsm_xxh3_128_stream_init_batch", "lsm_xxh3_128_stream_batch_workspace_size",
                    "lsm_xxh3_128_stream_update_batch", "lsm_xxh3_128_stream_digest_batch"]


def _check(rc, what):
    if rc != 0:
        raise LsmError(f"{what} failed: {STATUS.get(rc, rc)} {lib().lsm_last_error().decode()}")


def _torch():
    import torch
    if not torch.cuda.is_available():
        raise LsmError("no GPU visible: the lsmgpu product path has no CPU fallback")
    return torch


def _stream(stream):
    torch = _torch()
    s = stream if stream is not None else torch.cuda.current_stream()
    return C.c_void_p(s.cuda_stream)


def _ptr(t):
    return C.c_void_p(t.data_ptr()) if t is not None else None


def padded_bytes(n, device="cuda"):
    """uint8 device buffer of n bytes + LSM_INPUT_PADDING slack (16-aligned by the allocator)."""
    torch = _torch()
    buf = torch.zeros(n + LSM_INPUT_PADDING, dtype=torch.uint8, device=device)
    return buf


def to_device_bytes(data, device="cuda"):
    """Host bytes / numpy uint8 -> padded device buffer (first len bytes valid)."""
    import numpy as np
    torch = _torch()
    a = np.frombuffer(bytes(data), np.uint8) if isinstance(data, (bytes, bytearray, memoryview)) else np.asarray(data, np.uint8)
    buf = padded_bytes(len(a), device)
    if len(a):
        buf[:len(a)].copy_(torch.from_numpy(a.copy()))
    return buf


PARSED_FIELDS = (("seqno", "int64"), ("key_off", "int32"), ("val_off", "int32"), ("val_len", "int32"),
                 ("key_len", "int16"), ("prefix_len", "int16"), ("vtype", "uint8"), ("handle_off", "int64"))
# lsm_parsed_items16: 16-bit payload offsets and lengths, 19 B/item (no handle_off)
PARSED16_FIELDS = (("seqno", "int64"), ("key_off", "int16"), ("val_off", "int16"), ("val_len", "int16"),
                   ("key_len", "int16"), ("prefix_len", "int16"), ("vtype", "uint8"))


class Decoder:
    """Reusable decode context: holds the workspace for up to n_blocks."""

    def __init__(self, device="cuda"):
        self.device = device
        self.ws = None

    def workspace(self, n_blocks, blocks_bytes=0):
        """Workspace for n_blocks; with blocks_bytes (the batch buffer's size) it
        includes the pool that spreads blocks > 72 KiB over the whole GPU.  The
        cached buffer is returned viewed at exactly the size this call needs:
        the library turns the pool on from the size it is handed (lsmgpu.h), so
        bytes grown by an earlier pool call must not reach a pool=False call."""
        torch = _torch()
        need = (lib().lsm_decode_workspace_size_ex(n_blocks, blocks_bytes) if blocks_bytes
                else lib().lsm_decode_workspace_size(n_blocks))
        if self.ws is None or self.ws.numel() < need:
            self.ws = torch.empty(max(need, 256), dtype=torch.uint8, device=self.device)
        return self.ws[:need]

    def alloc_outputs(self, item_cap, n_blocks, fields=None, compact=False):
        torch = _torch()
        spec = PARSED16_FIELDS if compact else PARSED_FIELDS
        fields = fields or [f for f, _ in spec]
        out = {}
        for f, dt in spec:
            if f in fields:
                out[f] = torch.empty(max(item_cap, 1), dtype=getattr(torch, dt), device=self.device)
        out["item_start"] = torch.empty(n_blocks + 1, dtype=torch.int32, device=self.device)
        out["status"] = torch.empty(max(n_blocks, 1), dtype=torch.int32, device=self.device)
        return out

    def decode(self, blocks, block_off, n_blocks, out, item_cap, expect_type=-1, tuning=None, stream=None,
               compact=False, pool=None, workspace_bytes=None):
        """Enqueue lsm_decode_blocks (compact: lsm_decode_blocks16 into 16-bit
        offset arrays from alloc_outputs(..., compact=True)).  blocks: uint8 cuda
        (padded); block_off: int64 cuda [n+1].  pool=True: the workspace carries
        the pool that spreads blocks > 72 KiB over the GPU; False: the base
        workspace only (those blocks on one workgroup each); None (default): the
        pool when the batch's mean block is 32 KiB or more (its kernels cost a few
        microseconds per call even with no such block); workspace_bytes: pass
        exactly that much workspace (tests of a pool too small for the batch)."""
        if pool is None:
            pool = blocks.numel() >= HUGE_AUTO_MEAN * max(n_blocks, 1)
        if tuning is None and os.environ.get("LSMGPU_DECODE_TUNING"):  # diagnostic override
            tuning = tuple(int(x, 0) for x in os.environ["LSMGPU_DECODE_TUNING"].split(","))
        ws = self.workspace(n_blocks, blocks.numel() if pool else 0)
        if workspace_bytes is not None:
            ws = _torch().empty(max(workspace_bytes, 1), dtype=_torch().uint8, device=self.device)[:workspace_bytes]
        if compact:
            ps = LsmParsed16()
            for f, dt in PARSED16_FIELDS:
                if f in out and out[f].element_size() != C.sizeof(C.c_uint64 if dt == "int64" else
                                                                  C.c_uint16 if dt == "int16" else C.c_uint8):
                    raise LsmError(f"compact decode: field {f} must be {dt}")
                setattr(ps, f, out[f].data_ptr() if f in out else None)
            if pool:
                tuning = tuple(tuning or (0, 0, 0))
                tuning = tuning[:3] + ((tuning[3] if len(tuning) > 3 else 0) | DECODE_HUGE_POOL,)
            t = C.byref(LsmDecodeTuning(*tuning)) if tuning is not None else None
            rc = lib().lsm_decode_blocks16(_ptr(blocks), _ptr(block_off), n_blocks, expect_type, C.byref(ps),
                                           item_cap, _ptr(out["item_start"]), _ptr(out["status"]), _ptr(ws),
                                           ws.numel(), t, _stream(stream))
            _check(rc, "lsm_decode_blocks16")
            return out
        ps = LsmParsed()
        for f, _ in PARSED_FIELDS:
            setattr(ps, f, out[f].data_ptr() if f in out else None)
        if pool:  # the pool is an explicit opt-in (LSM_DECODE_HUGE_POOL), never implied by the size
            tuning = tuple(tuning or (0, 0, 0))
            tuning = tuning[:3] + ((tuning[3] if len(tuning) > 3 else 0) | DECODE_HUGE_POOL,)
        if tuning is not None:
            t = LsmDecodeTuning(*tuning)  # (blocks_per_wave, stage_bytes, tile_items[, flags])
            rc = lib().lsm_decode_blocks_tuned(_ptr(blocks), _ptr(block_off), n_blocks, expect_type, C.byref(ps),
                                               item_cap, _ptr(out["item_start"]), _ptr(out["status"]), _ptr(ws),
                                               ws.numel(), C.byref(t), _stream(stream))
        else:
            rc = lib().lsm_decode_blocks(_ptr(blocks), _ptr(block_off), n_blocks, expect_type, C.byref(ps), item_cap,
                                         _ptr(out["item_start"]), _ptr(out["status"]), _ptr(ws), ws.numel(),
                                         _stream(stream))
        _check(rc, "lsm_decode_blocks")
        return out


def decode_blocks(blocks, block_off, n_blocks=None, expect_type=-1, item_cap=None, fields=None, tuning=None,
                  compact=False, pool=None, workspace_bytes=None):
    """Convenience: decode device blocks, returns dict of device tensors
    (compact: the 19 B/item lsm_parsed_items16 layout)."""
    n_blocks = (block_off.numel() - 1) if n_blocks is None else n_blocks
    if item_cap is None:
        item_cap = blocks.numel() // 3 + 1
    d = Decoder(blocks.device)
    out = d.alloc_outputs(item_cap, n_blocks, fields, compact)
    return d.decode(blocks, block_off, n_blocks, out, item_cap, expect_type, tuning, compact=compact, pool=pool,
                    workspace_bytes=workspace_bytes)


class Encoder:
    def __init__(self, device="cuda"):
        self.device = device
        self.ws = None

    def encode(self, items, starts, n_blocks, restart_interval=16, hash_ratio=0.0, block_type=BLOCK_DATA,
               out=None, stream=None, pool=None, workspace_bytes=None, run_plan=False):
        """items: dict of cuda tensors keys(u8, padded) key_off(i64 n+1) vals(u8, padded) val_off(i64 n+1)
        seqno(i64) vtype(u8) [handle_off(i64) handle_size(i32)]; starts: int32 cuda [n_blocks+1].
        key_off / val_off as int32 tensors (arenas < 4 GiB): lsm_encode_blocks32 (u32 offsets).
        pool=False: the base workspace only (blocks > 96 KiB on one workgroup each);
        None (default): the pool when the output bound averages 32 KiB per block or more;
        workspace_bytes: pass exactly that much workspace (tests of a pool too small)."""
        torch = _torch()
        n_items = items["seqno"].numel()
        off32 = items["key_off"].element_size() == 4
        if off32 and "val_off" in items and items["val_off"].element_size() != 4:
            raise LsmError("key_off and val_off must have the same width")
        it = LsmItems32() if off32 else LsmItems()
        it.keys = items["keys"].data_ptr()
        it.key_off = items["key_off"].data_ptr()
        it.vals = items["vals"].data_ptr() if "vals" in items else items["keys"].data_ptr()
        it.val_off = items["val_off"].data_ptr() if "val_off" in items else items["key_off"].data_ptr()
        it.seqno = items["seqno"].data_ptr()
        it.vtype = items["vtype"].data_ptr() if "vtype" in items else None
        it.handle_off = items["handle_off"].data_ptr() if "handle_off" in items else None
        it.handle_size = items["handle_size"].data_ptr() if "handle_size" in items else None
        it.n_items = n_items
        params = LsmBlockParams(restart_interval, block_type, 0, 0, hash_ratio, 0)
        key_bytes = int(items["keys"].numel())
        val_bytes = int(items["vals"].numel()) if "vals" in items else 0
        bound = lib().lsm_encode_bound(n_items, n_blocks, key_bytes, val_bytes, C.byref(params))
        if pool is None:
            pool = bound >= HUGE_AUTO_MEAN * max(n_blocks, 1)
        if pool:  # the pool is an explicit opt-in (LSM_ENCODE_HUGE_POOL), never implied by the size
            params.flags = ENCODE_HUGE_POOL
        if run_plan:  # LSM_ENCODE_RUN_PLAN (the library also takes it by itself for long blocks)
            params.flags |= ENCODE_RUN_PLAN
        need = (lib().lsm_encode_workspace_size_ex(n_items, n_blocks, bound) if pool
                else lib().lsm_encode_workspace_size(n_items, n_blocks))
        if workspace_bytes is not None:
            need = workspace_bytes
        if self.ws is None or self.ws.numel() < need:
            self.ws = torch.empty(max(need, 256), dtype=torch.uint8, device=self.device)
        if out is None or out["buf"].numel() < bound:
            out = {"buf": torch.empty(bound + LSM_INPUT_PADDING, dtype=torch.uint8, device=self.device),
                   "block_off": torch.empty(n_blocks + 1, dtype=torch.int64, device=self.device),
                   "status": torch.empty(max(n_blocks, 1), dtype=torch.int32, device=self.device)}
        fn = lib().lsm_encode_blocks32 if off32 else lib().lsm_encode_blocks
        rc = fn(C.byref(it), _ptr(starts), n_blocks, C.byref(params), _ptr(out["buf"]), bound,
                _ptr(out["block_off"]), _ptr(out["status"]), _ptr(self.ws), need, _stream(stream))
        _check(rc, "lsm_encode_blocks32" if off32 else "lsm_encode_blocks")
        return out


def xxh3_128_batch(data, off, n):
    torch = _torch()
    out = torch.empty(2 * max(n, 1), dtype=torch.int64, device=data.device)
    _check(lib().lsm_xxh3_128_batch(_ptr(data), _ptr(off), n, _ptr(out), _stream(None)), "lsm_xxh3_128_batch")
    return out


def point_read(blocks, block_off, n_blocks, query_block, needles, needle_off, snapshot, stream=None):
    """Batched DataBlock::point_read (data_block/mod.rs:412-472).  All inputs cuda
    tensors: blocks uint8 (padded), block_off int64 [n_blocks+1], query_block
    int32 [n], needles uint8 (padded arena), needle_off int64 [n+1], snapshot
    int64 [n].  Returns dict item/seqno/val_off/val_len/vtype/status (item -1 = None)."""
    torch = _torch()
    n = int(query_block.numel())
    dev = blocks.device
    out = {"item": torch.empty(max(n, 1), dtype=torch.int32, device=dev),
           "seqno": torch.zeros(max(n, 1), dtype=torch.int64, device=dev),
           "val_off": torch.zeros(max(n, 1), dtype=torch.int32, device=dev),
           "val_len": torch.zeros(max(n, 1), dtype=torch.int32, device=dev),
           "vtype": torch.zeros(max(n, 1), dtype=torch.uint8, device=dev),
           "status": torch.empty(max(n, 1), dtype=torch.int32, device=dev)}
    res = LsmPointResult(*(_ptr(out[f]) for f in ("item", "seqno", "val_off", "val_len", "vtype")))
    _check(lib().lsm_point_read_blocks(_ptr(blocks), _ptr(block_off), n_blocks, _ptr(query_block), _ptr(needles),
                                       _ptr(needle_off), _ptr(snapshot), n, C.byref(res), _ptr(out["status"]),
                                       _stream(stream)), "lsm_point_read_blocks")
    return out


SEEK_LO, SEEK_HI, SEEK_LO_EXCLUSIVE, SEEK_HI_EXCLUSIVE = 1, 2, 4, 8


def seek(blocks, block_off, n_blocks, query_block, lo, lo_off, hi, hi_off, flags, stream=None):
    """Batched data_block::Iter::seek / seek_upper (+ exclusive) (data_block/iter.rs:37-176).
    All inputs cuda tensors: blocks uint8 (padded), block_off int64 [n_blocks+1], query_block
    int32 [n], lo / hi uint8 padded arenas with int64 [n+1] offsets, flags uint8 [n]
    (SEEK_* bits).  Returns dict first/end (int32: item range in block order), found
    (uint8: bit 0 lower, bit 1 upper seek's return value), status."""
    torch = _torch()
    n = int(query_block.numel())
    dev = blocks.device
    out = {"first": torch.empty(max(n, 1), dtype=torch.int32, device=dev),
           "end": torch.empty(max(n, 1), dtype=torch.int32, device=dev),
           "found": torch.empty(max(n, 1), dtype=torch.uint8, device=dev),
           "status": torch.empty(max(n, 1), dtype=torch.int32, device=dev)}
    _check(lib().lsm_seek_blocks(_ptr(blocks), _ptr(block_off), n_blocks, _ptr(query_block), _ptr(lo), _ptr(lo_off),
                                 _ptr(hi), _ptr(hi_off), _ptr(flags), n, _ptr(out["first"]), _ptr(out["end"]),
                                 _ptr(out["found"]), _ptr(out["status"]), _stream(stream)), "lsm_seek_blocks")
    return out


def xxh3_128_file(data, length=None, offset=0, stream=None):
    """Whole-file xxh3_128 (ChecksummedWriter digest) of data[offset .. offset+length)
    (uint8 cuda tensor, readable 16 B past the end) -> (low, high) as Python ints."""
    torch = _torch()
    length = data.numel() - offset if length is None else length
    ws = torch.empty(max(lib().lsm_xxh3_128_file_workspace_size(length), 256), dtype=torch.uint8, device=data.device)
    out = torch.zeros(2, dtype=torch.int64, device=data.device)
    _check(lib().lsm_xxh3_128_file(C.c_void_p(data.data_ptr() + offset), length, _ptr(out), _ptr(ws), ws.numel(),
                                   _stream(stream)), "lsm_xxh3_128_file")
    lo, hi = (int(x) & (2 ** 64 - 1) for x in out.cpu().tolist())
    return lo, hi


class ChecksummedWriter:
    """The running whole-file checksum of an SST writer (ChecksummedWriter,
    src/checksum.rs:59-96) with its state in device memory: write(data) feeds
    the next bytes (ChecksummedWriter::write, checksum.rs:92-95),
    checksum() is Xxh3Default::digest128 of everything written so far, as
    (low, high) Python ints (synchronises; the state is kept, writes may go on).
    Any split of the file into writes gives the one-shot xxh3_128.

    Every call runs on one stream, fixed at construction (`stream`, else the
    stream current then).  write() first makes that stream wait for the
    caller's current stream (where `data` was produced); checksum() waits for
    the digest on that stream before reading it back."""

    def __init__(self, device=None, stream=None):
        torch = _torch()
        self.device = torch.device("cuda") if device is None else torch.device(device)
        self.stream = stream if stream is not None else torch.cuda.current_stream(self.device)
        with torch.cuda.stream(self.stream):
            self.state = torch.empty(lib().lsm_xxh3_128_stream_state_size(), dtype=torch.uint8, device=self.device)
            self._ws = torch.empty(0, dtype=torch.uint8, device=self.device)
        self.bytes_written = 0
        _check(lib().lsm_xxh3_128_stream_init(_ptr(self.state), _stream(self.stream)), "lsm_xxh3_128_stream_init")

    def write(self, data, length=None, offset=0):
        """Feed data[offset .. offset + length) (uint8 cuda tensor, readable 16 B past the end)."""
        torch = _torch()
        length = data.numel() - offset if length is None else length
        cur = torch.cuda.current_stream(self.device)
        if cur != self.stream:
            self.stream.wait_stream(cur)           # data may still be being written on the caller's stream
            data.record_stream(self.stream)        # and must outlive the update queued below
        need = lib().lsm_xxh3_128_stream_workspace_size(length)
        if self._ws.numel() < need:
            # (allocated and freed on self.stream: the caching allocator reuses the old
            # workspace only for work queued after the updates that read it)
            with torch.cuda.stream(self.stream):
                self._ws = torch.empty(need, dtype=torch.uint8, device=self.device)
        _check(lib().lsm_xxh3_128_stream_update(_ptr(self.state), C.c_void_p(data.data_ptr() + offset), length,
                                                _ptr(self._ws), self._ws.numel(), _stream(self.stream)),
               "lsm_xxh3_128_stream_update")
        self.bytes_written += length
        return length

    def checksum(self):
        torch = _torch()
        with torch.cuda.stream(self.stream):
            out = torch.zeros(2, dtype=torch.int64, device=self.device)
        _check(lib().lsm_xxh3_128_stream_digest(_ptr(self.state), _ptr(out), _stream(self.stream)),
               "lsm_xxh3_128_stream_digest")
        self.stream.synchronize()
        lo, hi = (int(x) & (2 ** 64 - 1) for x in out.cpu().tolist())
        return lo, hi


class ChecksummedWriterSet:
    """n running whole-file checksums advanced together: one ChecksummedWriter
    (src/checksum.rs:59-96) per table of a flush or compaction that rotates
    through several tables (MultiWriter, src/table/multi_writer.rs:181-257).
    write(data, off) feeds state i the bytes data[off[i] .. off[i+1]) for every
    i in one launch sequence (lsm_xxh3_128_stream_update_batch); checksums()
    returns every digest as (low, high) pairs.  Same stream rules as
    ChecksummedWriter."""

    def __init__(self, n, device=None, stream=None):
        torch = _torch()
        self.n = n
        self.device = torch.device("cuda") if device is None else torch.device(device)
        self.stream = stream if stream is not None else torch.cuda.current_stream(self.device)
        size = lib().lsm_xxh3_128_stream_state_size()
        with torch.cuda.stream(self.stream):
            self.states = torch.empty(max(n, 1) * size, dtype=torch.uint8, device=self.device)
            self.status = torch.zeros(max(n, 1), dtype=torch.int32, device=self.device)
            self._ws = torch.empty(0, dtype=torch.uint8, device=self.device)
        _check(lib().lsm_xxh3_128_stream_init_batch(_ptr(self.states), n, _stream(self.stream)),
               "lsm_xxh3_128_stream_init_batch")

    def write(self, data, off, total_len=None):
        """data: uint8 cuda tensor (readable 16 B past each range); off: int64 cuda
        tensor [n+1]; total_len >= off[n] - off[0] (default: data.numel())."""
        torch = _torch()
        total_len = data.numel() if total_len is None else total_len
        cur = torch.cuda.current_stream(self.device)
        if cur != self.stream:
            self.stream.wait_stream(cur)
            data.record_stream(self.stream)
            off.record_stream(self.stream)
        need = lib().lsm_xxh3_128_stream_batch_workspace_size(self.n, total_len)
        if self._ws.numel() < need:
            with torch.cuda.stream(self.stream):
                self._ws = torch.empty(need, dtype=torch.uint8, device=self.device)
        _check(lib().lsm_xxh3_128_stream_update_batch(_ptr(self.states), self.n, _ptr(data), _ptr(off), total_len,
                                                      _ptr(self.status), _ptr(self._ws), self._ws.numel(),
                                                      _stream(self.stream)), "lsm_xxh3_128_stream_update_batch")
        return self.status

    def checksums(self):
        torch = _torch()
        with torch.cuda.stream(self.stream):
            out = torch.zeros(2 * max(self.n, 1), dtype=torch.int64, device=self.device)
        _check(lib().lsm_xxh3_128_stream_digest_batch(_ptr(self.states), self.n, _ptr(out), _stream(self.stream)),
               "lsm_xxh3_128_stream_digest_batch")
        self.stream.synchronize()
        v = [int(x) & (2 ** 64 - 1) for x in out.cpu().tolist()]
        return [(v[2 * i], v[2 * i + 1]) for i in range(self.n)]


BLOOM_BITS_PER_KEY, BLOOM_FP_RATE, BLOOM_BAD_FILTER = 0, 1, 0xFF


def bloom_shape(n, bpk=None, fpr=None):
    """BloomConstructionPolicy::{BitsPerKey, FalsePositiveRate}.init(n) -> (m, k)
    (src/table/filter/mod.rs:25-34).  Host-only."""
    m, k = C.c_uint64(), C.c_uint64()
    policy, value = (BLOOM_BITS_PER_KEY, bpk) if bpk is not None else (BLOOM_FP_RATE, fpr)
    _check(lib().lsm_bloom_shape(n, policy, value, C.byref(m), C.byref(k)), "lsm_bloom_shape")
    return m.value, k.value


def hash64_keys(keys, key_off, n=None, stream=None):
    """xxh3_64 of each key (FullFilterWriter::register_key, writer/filter/full.rs:47-50):
    keys = padded uint8 cuda tensor, key_off = int64 cuda tensor [n+1] -> int64 cuda [n]."""
    torch = _torch()
    n = key_off.numel() - 1 if n is None else n
    out = torch.empty(max(n, 1), dtype=torch.int64, device=keys.device)
    _check(lib().lsm_hash64_keys(_ptr(keys), _ptr(key_off), n, _ptr(out), _stream(stream)), "lsm_hash64_keys")
    return out[:n]


def bloom_build(hashes, m, k, stream=None):
    """Standard Bloom filter image (Builder::set_with_hash + build, standard_bloom/builder.rs)
    of int64 cuda hashes -> uint8 cuda tensor of lsm_bloom_filter_size(m) bytes."""
    torch = _torch()
    size = lib().lsm_bloom_filter_size(m)
    buf = torch.empty((size + 3) // 4 * 4, dtype=torch.uint8, device=hashes.device)
    _check(lib().lsm_bloom_build(_ptr(hashes), hashes.numel(), m, k, _ptr(buf), buf.numel(), _stream(stream)),
           "lsm_bloom_build")
    return buf[:size]


def bloom_contains(filt, hashes, stream=None):
    """contains_hash per hash (standard_bloom/mod.rs:100-120) -> uint8 cuda [n]: 1, 0 or BLOOM_BAD_FILTER."""
    torch = _torch()
    out = torch.empty(max(hashes.numel(), 1), dtype=torch.uint8, device=hashes.device)
    _check(lib().lsm_bloom_contains(_ptr(filt), filt.numel(), _ptr(hashes), hashes.numel(), _ptr(out),
                                    _stream(stream)), "lsm_bloom_contains")
    return out[:hashes.numel()]


# Default cap on a header's uncompressed_length (the plan sizes the output from
# verified headers only, but a crafted header per block could still ask for
# this much): the writer's largest data-block target is 4 MiB
# (writer/mod.rs:195-198) and a block overshoots its target by its last item
# (mod.rs:284-290), so 4 MiB + 64 KiB covers tables of items < 64 KiB; pass a
# larger max_block_bytes for tables with larger items.
LZ4_MAX_BLOCK = (4 << 20) + (64 << 10)


def lz4_decompress_blocks(blocks, block_off, n_blocks=None, max_block_bytes=LZ4_MAX_BLOCK, stream=None):
    """Block::from_reader with CompressionType::Lz4 over a batch (block/mod.rs:87-128):
    blocks = padded uint8 cuda tensor of on-disk blocks, block_off = int64 cuda [n+1].
    Output sizes come from lsm_lz4_plan_output: each VERIFIED header's
    uncompressed_length (a block whose header fails gets 0 bytes and reports the
    header error; one above max_block_bytes reports OVERFLOW).
    Returns (out uint8 cuda, out_off int64 cuda [n+1], status int32 cuda [n])."""
    torch = _torch()
    n = block_off.numel() - 1 if n_blocks is None else n_blocks
    dev = blocks.device
    out_off = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    if n:
        pws = torch.empty(lib().lsm_lz4_plan_workspace_size(n), dtype=torch.uint8, device=dev)
        _check(lib().lsm_lz4_plan_output(_ptr(blocks), _ptr(block_off), n, max_block_bytes, _ptr(out_off), _ptr(pws),
                                         pws.numel(), _stream(stream)), "lsm_lz4_plan_output")
    total = int(out_off[-1].item()) if n else 0
    out = torch.empty(max(total, 1), dtype=torch.uint8, device=dev)
    status = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
    ws = torch.empty(lib().lsm_lz4_workspace_size(n), dtype=torch.uint8, device=dev)
    _check(lib().lsm_lz4_decompress_blocks(_ptr(blocks), _ptr(block_off), n, _ptr(out), _ptr(out_off),
                                           _ptr(status), _ptr(ws), ws.numel(), _stream(stream)),
           "lsm_lz4_decompress_blocks")
    return out, out_off, status[:n]


def decode_lz4_blocks(blocks, block_off, n_blocks=None, expect_type=-1, item_cap=None, fields=None,
                      max_block_bytes=LZ4_MAX_BLOCK, stream=None, frames_cap=None):
    """LZ4 blocks end to end: Block::from_reader(Lz4) then DataBlock::new + iter
    (block/mod.rs:104-118, data_block/mod.rs:335,476).  lsm_lz4_plan_framed ->
    lsm_lz4_decompress_framed (frames = Header' || decompressed payload) ->
    lsm_decode_blocks_tuned(frames, LSM_DECODE_PAYLOAD_VERIFIED).  Returns the decode
    output dict (payload-relative offsets into each frame's payload) plus "frames",
    "frame_off" and "status" = the decompress status where it is not OK, else the
    decode status ("decode_status": the decode's own statuses: a block whose
    decompression failed has an all-zero frame header, so it is BAD_MAGIC there
    even without the merge).  frames_cap (bytes): size the frame arena without
    reading the plan back (no host sync; every block whose header verifies reports
    LSM_OVERFLOW when the frames do not fit, and item_cap defaults to frames_cap // 3)."""
    torch = _torch()
    n = block_off.numel() - 1 if n_blocks is None else n_blocks
    dev = blocks.device
    frame_off = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    if n:
        pws = torch.empty(lib().lsm_lz4_plan_workspace_size(n), dtype=torch.uint8, device=dev)
        if frames_cap is not None:
            _check(lib().lsm_lz4_plan_capped(_ptr(blocks), _ptr(block_off), n, max_block_bytes, 1, frames_cap,
                                             _ptr(frame_off), _ptr(pws), pws.numel(), _stream(stream)),
                   "lsm_lz4_plan_capped")
        else:
            _check(lib().lsm_lz4_plan_framed(_ptr(blocks), _ptr(block_off), n, max_block_bytes, _ptr(frame_off),
                                             _ptr(pws), pws.numel(), _stream(stream)), "lsm_lz4_plan_framed")
    if frames_cap is not None:
        total = frames_cap
    else:
        total = int(frame_off[-1].item()) if n else 0
    frames = padded_bytes(total, dev)
    zst = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
    ws = torch.empty(lib().lsm_lz4_workspace_size(n), dtype=torch.uint8, device=dev)
    _check(lib().lsm_lz4_decompress_framed(_ptr(blocks), _ptr(block_off), n, _ptr(frames), _ptr(frame_off),
                                           _ptr(zst), _ptr(ws), ws.numel(), _stream(stream)),
           "lsm_lz4_decompress_framed")
    if item_cap is None:
        item_cap = total // 3 + 1
    d = Decoder(dev)
    out = d.alloc_outputs(item_cap, n, fields)
    d.decode(frames, frame_off, n, out, item_cap, expect_type,
             tuning=(0, 0, 0, DECODE_PAYLOAD_VERIFIED), stream=stream)
    out["decode_status"] = out["status"].clone()  # (what a caller sees without the merge below)
    out["status"] = torch.where(zst[:max(n, 1)] != 0, zst[:max(n, 1)], out["status"])
    out["frames"], out["frame_off"] = frames, frame_off
    return out


def materialize_keys(blocks, block_off, n_blocks, out, n_items=None, stream=None, key_cap=None):
    """DataBlockParsedItem::materialize (data_block/mod.rs:296-315) of decode output `out`
    (dict from decode_blocks / scan_table) -> (keys uint8 cuda arena, key_off int64 cuda
    [n_items+1]); values stay (val_off, val_len) sub-slices of each payload.
    key_cap (bytes): no host sync (n_items defaults to the parsed arrays' capacity,
    lsm_materialize_keys_capped); returns (keys, key_off, result) with result a
    device int32 [1]: LSM_OK, or LSM_OVERFLOW when the keys exceed key_cap (none written)."""
    torch = _torch()
    dev = blocks.device
    if n_items is None:
        n_items = out["key_off"].numel() if key_cap is not None else int(out["item_start"][n_blocks].item())
    key_off = torch.zeros(n_items + 1, dtype=torch.int64, device=dev)
    ps = LsmParsed()
    for f, _ in PARSED_FIELDS:
        setattr(ps, f, out[f].data_ptr() if f in out else None)
    ws = torch.empty(lib().lsm_materialize_workspace_size(n_items), dtype=torch.uint8, device=dev)
    args = (_ptr(blocks), _ptr(block_off), n_blocks, _ptr(out["item_start"]), _ptr(out["status"]), C.byref(ps), n_items)
    _check(lib().lsm_materialize_plan(*args, _ptr(key_off), _ptr(ws), ws.numel(), _stream(stream)),
           "lsm_materialize_plan")
    if key_cap is not None:
        keys = padded_bytes(key_cap, dev)
        result = torch.empty(1, dtype=torch.int32, device=dev)
        _check(lib().lsm_materialize_keys_capped(*args, _ptr(key_off), _ptr(keys), key_cap, _ptr(result),
                                                 _stream(stream)), "lsm_materialize_keys_capped")
        return keys, key_off, result
    total = int(key_off[-1].item()) if n_items else 0
    keys = padded_bytes(total, dev)
    _check(lib().lsm_materialize_keys(*args, _ptr(key_off), _ptr(keys), _stream(stream)), "lsm_materialize_keys")
    return keys, key_off


def scan_table(file, file_len, tli_off, tli_size, two_level=False, global_seqno=0, block_count=0, cap_blocks=None,
               item_cap=None, fields=None, stream=None, sync=True, data_blocks_hint=0, index_blocks_hint=0):
    """Scanner over a table file image (scanner.rs:24-92): file = padded uint8 cuda tensor.
    Returns dict: table_status (int), n_blocks (int), block_off (int64 cuda [n+1]),
    the parsed fields, item_start and status (as decode_blocks).
    sync=False: lsm_scan_table_async (no host synchronisation): table_status and
    n_blocks are device int32 / uint32 tensors of one element, block_off holds
    cap_blocks + 1 entries (data_blocks_hint bounds the data decode, e.g. block_count;
    index_blocks_hint the partitions of a two-level index, e.g. tli_size // 4)."""
    torch = _torch()
    dev = file.device
    if cap_blocks is None:
        cap_blocks = max(1, file_len // 33)
    if item_cap is None:
        item_cap = file_len // 3 + 1
    out = Decoder(dev).alloc_outputs(item_cap, cap_blocks, fields)
    block_off = torch.zeros(cap_blocks + 1, dtype=torch.int64, device=dev)
    ws = torch.empty(lib().lsm_scan_workspace_size(cap_blocks), dtype=torch.uint8, device=dev)
    ps = LsmParsed()
    for f, _ in PARSED_FIELDS:
        setattr(ps, f, out[f].data_ptr() if f in out else None)
    t = LsmTableScan(tli_off, tli_size, int(bool(two_level)), global_seqno & (2 ** 64 - 1), block_count)
    if not sync:
        d_nb = torch.zeros(1, dtype=torch.int32, device=dev)
        d_ts = torch.zeros(1, dtype=torch.int32, device=dev)
        _check(lib().lsm_scan_table_async(_ptr(file), file_len, C.byref(t), _ptr(block_off), cap_blocks,
                                          index_blocks_hint, data_blocks_hint, C.byref(ps), item_cap, _ptr(out["item_start"]),
                                          _ptr(out["status"]), _ptr(d_nb), _ptr(d_ts), _ptr(ws), ws.numel(),
                                          _stream(stream)), "lsm_scan_table_async")
        out["table_status"], out["n_blocks"], out["block_off"] = d_ts, d_nb, block_off
        return out
    nb, tst = C.c_uint32(), C.c_int32()
    _check(lib().lsm_scan_table(_ptr(file), file_len, C.byref(t), _ptr(block_off), cap_blocks, C.byref(ps), item_cap,
                                _ptr(out["item_start"]), _ptr(out["status"]), C.byref(nb), C.byref(tst), _ptr(ws),
                                ws.numel(), _stream(stream)), "lsm_scan_table")
    out["table_status"], out["n_blocks"] = int(tst.value), int(nb.value)
    out["block_off"] = block_off[:nb.value + 1]
    return out


def cut_blocks(key_off, val_off, block_size):
    """Host-side Writer chunking (numpy uint64 [n+1] arrays) -> numpy uint32 starts."""
    import numpy as np
    key_off = np.ascontiguousarray(key_off, np.uint64)
    val_off = np.ascontiguousarray(val_off, np.uint64)
    n = len(key_off) - 1
    starts = np.zeros(n + 2, np.uint32)
    nb = lib().lsm_cut_blocks(key_off.ctypes.data, val_off.ctypes.data, n, block_size, starts.ctypes.data, n + 1)
    return starts[:nb + 1].copy()


def items_to_device(items_np, device="cuda", off32=False):
    """pyoracle.Items-like numpy SoA -> dict of padded cuda tensors for Encoder.encode
    (off32: int32 key / value offsets, encoded through lsm_encode_blocks32)."""
    import numpy as np
    torch = _torch()
    d = {"keys": to_device_bytes(items_np.keys, device), "vals": to_device_bytes(items_np.vals, device)}
    ot = np.int32 if off32 else np.int64
    if off32 and (int(items_np.key_off[-1]) >= 1 << 32 or int(items_np.val_off[-1]) >= 1 << 32):
        raise LsmError("off32: arenas of 4 GiB or more need the u64 offsets")
    d["key_off"] = torch.from_numpy(items_np.key_off.astype(np.uint32 if off32 else np.int64).view(ot)).to(device)
    d["val_off"] = torch.from_numpy(items_np.val_off.astype(np.uint32 if off32 else np.int64).view(ot)).to(device)
    d["seqno"] = torch.from_numpy(items_np.seqno.view(np.int64)).to(device)
    d["vtype"] = torch.from_numpy(items_np.vtype).to(device)
    d["handle_off"] = torch.from_numpy(items_np.handle_off.view(np.int64)).to(device)
    d["handle_size"] = torch.from_numpy(items_np.handle_size.view(np.int32)).to(device)
    return d


def shard_blocks(block_off, world):
    """Split n blocks into `world` contiguous shards of about equal BYTES
    (blocks are independent, so shards need no exchange).
    block_off: host array-like of n+1 offsets.  Returns world+1 block indices
    b[0]=0 <= b[1] <= ... <= b[world]=n; rank r decodes blocks [b[r], b[r+1])."""
    import numpy as np
    off = np.asarray(block_off, dtype=np.uint64)
    n = len(off) - 1
    total = int(off[-1] - off[0])
    bounds = [0]
    for r in range(1, world):
        target = int(off[0]) + total * r // world
        b = int(np.searchsorted(off[:n], np.uint64(target), side="left"))
        bounds.append(max(bounds[-1], min(b, n)))
    bounds.append(n)
    return bounds


def shard_items(starts, key_off, val_off, world):
    """Encode-side split: `world` contiguous block ranges,
    cut only at block boundaries, of about equal key + value BYTES.
    starts: host [n_blocks+1] item starts; key_off / val_off: host [n_items+1].
    Returns world+1 block indices (as shard_blocks)."""
    import numpy as np
    st = np.asarray(starts, dtype=np.int64)
    w = np.asarray(key_off, dtype=np.uint64)[st] + np.asarray(val_off, dtype=np.uint64)[st]
    return shard_blocks(w, world)


def _dev_items(items, i0, i1, device):
    """Items [i0, i1) of a host SoA (pyoracle.Items layout) as rebased, padded device tensors."""
    import numpy as np
    torch = _torch()
    k0, k1 = int(items.key_off[i0]), int(items.key_off[i1])
    v0, v1 = int(items.val_off[i0]), int(items.val_off[i1])
    d = {"keys": to_device_bytes(items.keys[k0:k1], device), "vals": to_device_bytes(items.vals[v0:v1], device)}
    d["key_off"] = torch.from_numpy((items.key_off[i0:i1 + 1] - np.uint64(k0)).astype(np.int64)).to(device)
    d["val_off"] = torch.from_numpy((items.val_off[i0:i1 + 1] - np.uint64(v0)).astype(np.int64)).to(device)
    d["seqno"] = torch.from_numpy(np.ascontiguousarray(items.seqno[i0:i1]).view(np.int64)).to(device)
    d["vtype"] = torch.from_numpy(np.ascontiguousarray(items.vtype[i0:i1])).to(device)
    d["handle_off"] = torch.from_numpy(np.ascontiguousarray(items.handle_off[i0:i1]).view(np.int64)).to(device)
    d["handle_size"] = torch.from_numpy(np.ascontiguousarray(items.handle_size[i0:i1]).view(np.int32)).to(device)
    return d


def _pinned(arr):
    """A host numpy array copied into page-locked memory (torch tensor; the copy
    runs in numpy, which releases the GIL for it)."""
    import numpy as np
    torch = _torch()
    a = np.ascontiguousarray(arr)
    t = torch.empty(a.nbytes, dtype=torch.uint8, pin_memory=True)
    if a.nbytes:
        np.copyto(t.numpy(), a.view(np.uint8).reshape(-1))
    return t


def _run_shards(jobs, worker):
    """One host thread per shard (each drives its own device and stream; the
    library calls and torch copies release the GIL), with a barrier for the one
    exchange step.  worker(k, job, barrier) -> result; a failing shard aborts
    the barrier so no other shard waits forever, and its exception is raised."""
    import threading
    from concurrent.futures import ThreadPoolExecutor
    if not jobs:
        return []
    barrier = threading.Barrier(len(jobs))

    def run(k):
        try:
            return worker(k, jobs[k], barrier)
        except BaseException:
            barrier.abort()
            raise
    with ThreadPoolExecutor(max_workers=len(jobs)) as ex:
        futs = [ex.submit(run, k) for k in range(len(jobs))]
        return [f.result() for f in futs]


def encode_sharded(items, starts, devices, restart_interval=16, hash_ratio=0.0, block_type=BLOCK_DATA):
    """Single-process multi-device encode:
    the blocks of a host write buffer (pyoracle.Items layout, starts [n+1]) are
    split into len(devices) contiguous shards at block cuts (shard_items).  One
    host thread per shard: it stages the shard's items in pinned memory, copies
    them to its device on its own stream, encodes there and reads back the
    shard's block offsets; the one exchange step is the exclusive scan of the
    shards' byte totals (a barrier across the threads), after which every
    thread copies its blocks asynchronously into its place in one pinned packed
    buffer.  Shards overlap end to end (no blocking copy serialises them).
    Returns (packed bytes, block_off [n+1], status [n]) as host numpy arrays,
    equal to a single-device encode."""
    import numpy as np
    torch = _torch()
    starts = np.asarray(starts, dtype=np.int64)
    n_blocks = len(starts) - 1
    bounds = shard_items(starts, items.key_off, items.val_off, len(devices))
    jobs = [(dev, bounds[r], bounds[r + 1]) for r, dev in enumerate(devices) if bounds[r + 1] > bounds[r]]
    totals = [0] * len(jobs)
    shared = {}

    def worker(k, job, barrier):
        dev, b0, b1 = job
        dev = torch.device("cuda", dev) if isinstance(dev, int) else torch.device(dev)
        torch.cuda.set_device(dev)
        i0, i1 = int(starts[b0]), int(starts[b1])
        k0, k1 = int(items.key_off[i0]), int(items.key_off[i1])
        v0, v1 = int(items.val_off[i0]), int(items.val_off[i1])
        host = {"keys": _pinned(items.keys[k0:k1]), "vals": _pinned(items.vals[v0:v1]),
                "key_off": _pinned((items.key_off[i0:i1 + 1] - np.uint64(k0)).astype(np.int64)),
                "val_off": _pinned((items.val_off[i0:i1 + 1] - np.uint64(v0)).astype(np.int64)),
                "seqno": _pinned(items.seqno[i0:i1]), "vtype": _pinned(items.vtype[i0:i1]),
                "starts": _pinned((starts[b0:b1 + 1] - i0).astype(np.int32))}
        if items.handle_off is not None:
            host["handle_off"] = _pinned(items.handle_off[i0:i1])
            host["handle_size"] = _pinned(items.handle_size[i0:i1])
        st = torch.cuda.Stream(dev)
        nb = b1 - b0
        with torch.cuda.stream(st):
            d = {}
            for name, dt in (("keys", torch.uint8), ("vals", torch.uint8), ("key_off", torch.int64),
                             ("val_off", torch.int64), ("seqno", torch.int64), ("vtype", torch.uint8),
                             ("handle_off", torch.int64), ("handle_size", torch.int32)):
                if name not in host:
                    continue
                h = host[name].view(dt)
                if name in ("keys", "vals"):
                    t = padded_bytes(h.numel(), dev)
                    t[:h.numel()].copy_(h, non_blocking=True)
                else:
                    t = torch.empty(h.numel(), dtype=dt, device=dev)
                    t.copy_(h, non_blocking=True)
                d[name] = t
            d_starts = torch.empty(nb + 1, dtype=torch.int32, device=dev)
            d_starts.copy_(host["starts"].view(torch.int32), non_blocking=True)
            enc = Encoder(dev).encode(d, d_starts, nb, restart_interval, hash_ratio, block_type, stream=st)
            off_h = torch.empty(nb + 1, dtype=torch.int64, pin_memory=True)
            st_h = torch.empty(nb, dtype=torch.int32, pin_memory=True)
            off_h.copy_(enc["block_off"][:nb + 1], non_blocking=True)
            st_h.copy_(enc["status"][:nb], non_blocking=True)
        st.synchronize()
        totals[k] = int(off_h[-1])
        barrier.wait()  # exchange: every shard's byte total is known
        if k == 0:
            shared["packed"] = torch.empty(sum(totals), dtype=torch.uint8, pin_memory=True)
        barrier.wait()
        base = sum(totals[:k])
        with torch.cuda.stream(st):
            if totals[k]:
                shared["packed"][base:base + totals[k]].copy_(enc["buf"][:totals[k]], non_blocking=True)
        st.synchronize()
        off = off_h.numpy().view(np.uint64)
        return off[1:] + np.uint64(base), st_h.numpy().copy()

    res = _run_shards(jobs, worker)
    packed = shared["packed"].numpy() if jobs else np.zeros(0, np.uint8)
    block_off = np.concatenate([np.zeros(1, np.uint64)] + [r[0] for r in res])
    status = np.concatenate([r[1] for r in res]) if res else np.zeros(0, np.int32)
    assert len(block_off) == n_blocks + 1
    return packed, block_off, status


def decode_sharded(blocks, block_off, devices, expect_type=-1, fields=None):
    """Single-process multi-device decode: the on-disk blocks
    of a host buffer (e.g. an mmap'd SST's data section; block_off [n+1]) are
    split into len(devices) byte-balanced contiguous shards (shard_blocks).  One
    host thread per shard stages its bytes in pinned memory, copies them to its
    device on its own stream and decodes there; after the exchange step (the
    exclusive scan of the shards' item totals, a barrier across the threads)
    each thread copies its rows asynchronously into one pinned gather buffer
    per field, item_start rebased.  Returns host numpy arrays: every requested
    field, item_start [n+1] and status [n]."""
    import numpy as np
    torch = _torch()
    boff = np.asarray(block_off, dtype=np.uint64)
    data = np.frombuffer(blocks, np.uint8) if isinstance(blocks, (bytes, bytearray, memoryview)) else \
        np.asarray(blocks, np.uint8)
    n_blocks = len(boff) - 1
    bounds = shard_blocks(boff, len(devices))
    fields = fields or [f for f, _ in PARSED_FIELDS]
    jobs = [(dev, bounds[r], bounds[r + 1]) for r, dev in enumerate(devices) if bounds[r + 1] > bounds[r]]
    counts = [0] * len(jobs)
    shared = {}

    def worker(k, job, barrier):
        dev, b0, b1 = job
        dev = torch.device("cuda", dev) if isinstance(dev, int) else torch.device(dev)
        torch.cuda.set_device(dev)
        o0, o1 = int(boff[b0]), int(boff[b1])
        nb = b1 - b0
        hb = _pinned(data[o0:o1])
        ho = _pinned((boff[b0:b1 + 1] - np.uint64(o0)).astype(np.int64))
        st = torch.cuda.Stream(dev)
        cap = (o1 - o0) // 3 + 1
        with torch.cuda.stream(st):
            d_blocks = padded_bytes(o1 - o0, dev)
            d_blocks[:o1 - o0].copy_(hb, non_blocking=True)
            d_off = torch.empty(nb + 1, dtype=torch.int64, device=dev)
            d_off.copy_(ho.view(torch.int64), non_blocking=True)
            dec = Decoder(dev)
            out = dec.alloc_outputs(cap, nb, fields)
            dec.decode(d_blocks, d_off, nb, out, cap, expect_type, stream=st)
            ist_h = torch.empty(nb + 1, dtype=torch.int32, pin_memory=True)
            st_h = torch.empty(nb, dtype=torch.int32, pin_memory=True)
            ist_h.copy_(out["item_start"][:nb + 1], non_blocking=True)
            st_h.copy_(out["status"][:nb], non_blocking=True)
        st.synchronize()
        ist = ist_h.numpy().view(np.uint32).astype(np.int64)
        counts[k] = int(ist[-1])
        barrier.wait()  # exchange: every shard's item total is known
        if k == 0:
            tot = sum(counts)
            shared.update({f: torch.empty(max(tot, 1), dtype=out[f].dtype, pin_memory=True) for f in fields})
        barrier.wait()
        base = sum(counts[:k])
        with torch.cuda.stream(st):
            if counts[k]:
                for f in fields:
                    shared[f][base:base + counts[k]].copy_(out[f][:counts[k]], non_blocking=True)
        st.synchronize()
        return ist[1:] + base, st_h.numpy().copy()

    res_sh = _run_shards(jobs, worker)
    total = sum(counts)
    res = {f: (shared[f][:total].numpy() if jobs else np.zeros(0)) for f in fields}
    res["item_start"] = np.concatenate([np.zeros(1, np.int64)] + [r[0] for r in res_sh])
    res["status"] = np.concatenate([r[1] for r in res_sh]) if res_sh else np.zeros(0, np.int32)
    assert len(res["item_start"]) == n_blocks + 1
    return res
