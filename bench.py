#!/usr/bin/env python3
"""bench.py — BASELINE.json headline: "device-resident data-block decode+encode
GiB/s, 1 M x 4 KiB blocks" (configs[1] shape, configs[2] round trip).

A "step" is one pass of the hot path over the batch, both directions:
  lsm_encode_blocks   the item SoA (keys, values, seqnos, types) of 1 M blocks
                      -> on-disk blocks (DataBlock::encode_into + Block::write_into,
                      payload xxh3_128 + header fused), then
  lsm_decode_blocks   those blocks -> verified + parsed item SoA (Block::from_file
                      + DataBlock::iter: trailer counts, scan, header / xxh3_128
                      verify, full parse).
Inputs are resident in HBM when the timed region starts; nothing is cached
between steps (every step re-encodes and re-decodes the whole batch).
value = block bytes that went through encode AND decode, all ranks, per second
      = N_ranks x block_bytes x K / (max over ranks of the timed K steps).
(SURVEY §8(d) counts a round trip as W_enc + R_dec = 2 x block_bytes; that
figure is reported as `round_trip_traffic_GiB_per_s`, never as `value`.)

Synthetic input: keys = 16 B big-endian counters, values 64 B
uniform random, seqno 63, all Value, cut by the writer rule at 4096 B (52 items /
3769-3773 B per block), restart interval 16, hash ratio 0.  Outside the timed
region EVERY block is checked: encoded bytes == the oracle's encode (memcmp),
decoded fields == the oracle's decode (multithreaded oracle on the host).

N > 1: one process per GPU (torch.distributed, RCCL only for the max-time /
byte-sum reductions), each rank round-trips its own 1 M-block batch (weak
scaling, no data-path collective).

Also in the same JSON line (not `value`): per-kernel rooflines (decode, encode)
with the measured copy / LDS-DMA read ceilings, configs[3] (prefix-heavy 16 KiB),
configs[4] (8 GiB mixed 4/16/64 KiB data + index blocks byte-split across ranks),
point reads, range seeks, whole-file checksum, Bloom filter, LZ4 (and the
LZ4 -> parse chain), device materialize, a whole-table scan, the
host-inclusive rates (decode from an mmap'd file, encode from a host write
buffer) and the CPU baseline (oracle port on the host cores, 1 thread and all).
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import mmap
import os
import sys
import tempfile
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
for p in (ROOT / "lsm-tree_amd", ROOT / "oracle", ROOT / "tests"):
    sys.path.insert(0, str(p))

BASELINE_METRIC = "device-resident data-block decode+encode GiB/s, 1 M × 4 KiB blocks"  # BASELINE.json
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec, /opt/skills/guides/MI355X_MICROARCH.md
PARSED_BYTES_PER_ITEM = 8 + 4 + 4 + 4 + 2 + 2 + 1  # seqno key_off val_off val_len key_len prefix_len vtype
PER_BLOCK_OUT = 8  # item_start u32 + status i32
# encode input per item as the ABI reads it: key + value bytes, seqno u64, vtype u8, key_off / val_off u64
ENC_IN_PER_ITEM = 8 + 1 + 8 + 8
# the same as SURVEY §8(d) counts it: 4-byte key / value offsets
ENC_IN_PER_ITEM_SURVEY = 8 + 1 + 4 + 4
DATA_FIELDS = ["seqno", "key_off", "val_off", "val_len", "key_len", "prefix_len", "vtype"]
FIELD_NP = {"seqno": "uint64", "key_off": "uint32", "val_off": "uint32", "val_len": "uint32", "key_len": "uint16",
            "prefix_len": "uint16", "vtype": "uint8", "handle_off": "uint64"}
HOST_THREADS = 16  # the GPU box's CPU share per GPU (nproc shows the whole machine)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def host_threads(world=1):
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    # each rank's share of the machine, at most the per-GPU CPU share
    return max(1, min(HOST_THREADS, n // max(1, world)))


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


# ---------------------------------------------------------------- workloads
def make_workload(torch, lsmgpu, n_blocks, items_per_block=52, key_len=16, val_len=64, seed=0x5EED0002,
                  kind="counter"):
    """Synthetic items on the GPU, cut every items_per_block items (= the writer
    rule for these fixed sizes, check_cut_rule).  kind: "counter" = big-endian
    counter keys (G1); "prefix" = fixed random (key_len - 8)-byte prefix || 8-byte
    BE counter (config 4); "random" = random 16-byte keys, sorted (G2)."""
    dev = "cuda"
    n = n_blocks * items_per_block
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    ctr = torch.arange(n, dtype=torch.int64, device=dev)
    keys = torch.zeros(n * key_len + lsmgpu.LSM_INPUT_PADDING, dtype=torch.uint8, device=dev)
    kv = keys[:n * key_len].view(n, key_len)
    if kind == "random":
        assert key_len == 16
        hi = torch.randint(0, 1 << 62, (n,), dtype=torch.int64, device=dev, generator=g).sort().values
        lo = torch.randint(0, 1 << 62, (n,), dtype=torch.int64, device=dev, generator=g)
        kv[:, :8] = hi.view(torch.uint8).view(n, 8).flip(1)
        kv[:, 8:] = lo.view(torch.uint8).view(n, 8).flip(1)
    else:
        if kind == "prefix":
            kv[:, :key_len - 8] = torch.randint(0, 256, (key_len - 8,), dtype=torch.uint8, device=dev, generator=g)
        kv[:, key_len - 8:] = ctr.view(torch.uint8).view(n, 8).flip(1)
    vals = torch.randint(0, 256, (n * val_len + lsmgpu.LSM_INPUT_PADDING,), dtype=torch.uint8, device=dev,
                         generator=g)
    items = {
        "keys": keys,
        "key_off": torch.arange(n + 1, dtype=torch.int64, device=dev) * key_len,
        "vals": vals,
        "val_off": torch.arange(n + 1, dtype=torch.int64, device=dev) * val_len,
        "seqno": torch.full((n,), 63, dtype=torch.int64, device=dev),
        "vtype": torch.zeros(n, dtype=torch.uint8, device=dev),
    }
    starts = (torch.arange(n_blocks + 1, dtype=torch.int64, device=dev) * items_per_block).to(torch.int32)
    return items, starts, n


def check_cut_rule(lsmgpu, items_per_block, key_len, val_len, block_size=4096):
    """The fixed-count cut equals the reference writer rule (writer/mod.rs:284-290)."""
    import numpy as np
    m = items_per_block * 4
    ko = np.arange(m + 1, dtype=np.uint64) * key_len
    vo = np.arange(m + 1, dtype=np.uint64) * val_len
    starts = lsmgpu.cut_blocks(ko, vo, block_size)
    assert list(starts) == list(range(0, m + 1, items_per_block)), starts


# ------------------------------------------------------- full oracle checks
def host_items(items, n):
    """Device item SoA -> pyoracle.Items over host copies (no dtype copies)."""
    import numpy as np
    import pyoracle
    ko = items["key_off"][:n + 1].cpu().numpy().view(np.uint64)
    vo = items["val_off"][:n + 1].cpu().numpy().view(np.uint64) if "val_off" in items else np.zeros(n + 1, np.uint64)
    kb = items["keys"][:int(ko[-1])].cpu().numpy()
    vb = items["vals"][:int(vo[-1])].cpu().numpy() if "vals" in items else np.zeros(1, np.uint8)
    seq = items["seqno"][:n].cpu().numpy().view(np.uint64)
    vt = items["vtype"][:n].cpu().numpy() if "vtype" in items else np.zeros(n, np.uint8)
    ho = items["handle_off"][:n].cpu().numpy().view(np.uint64) if "handle_off" in items else None
    hs = items["handle_size"][:n].cpu().numpy().view(np.uint32) if "handle_size" in items else None
    return pyoracle.Items(kb, ko, vb, vo, seq, vt, ho, hs)


def check_encode_all(torch, items, starts, enc, nb, n_items, threads, restart_interval=16, block_type=0,
                     hash_ratio=0.0):
    """Every encoded block == the oracle's DataBlock::encode_into + Block::write_into
    of the same items (one memcmp over the whole batch).  Returns (ref_buf, ref_off)."""
    import numpy as np
    import pyoracle
    assert int((enc["status"][:nb] != 0).sum().item()) == 0, "encode status"
    it = host_items(items, n_items)
    st = starts[:nb + 1].cpu().numpy().astype(np.uint32)
    ref_buf, ref_off = pyoracle.encode_blocks(it, st, restart_interval=restart_interval, block_type=block_type,
                                              hash_ratio=hash_ratio, nthreads=threads)
    got_off = enc["block_off"][:nb + 1].cpu().numpy().view(np.uint64)
    assert np.array_equal(got_off, ref_off), "block offsets differ from the oracle"
    got = enc["buf"][:int(ref_off[-1])].cpu().numpy()
    assert np.array_equal(got, ref_buf), "encoded bytes differ from the oracle"
    return ref_buf, ref_off


def check_decode_all(dec, ref_buf, ref_off, nb, threads, fields=DATA_FIELDS, expect_status_ok=True):
    """Every block's status, item_start and every parsed field == the oracle's
    Block::from_file + full forward DataBlock::iter / IndexBlock::iter."""
    import numpy as np
    import pyoracle
    n_est = int(dec["item_start"][nb].item())
    parsed, item_start, status = pyoracle.decode_blocks(ref_buf, ref_off, nthreads=threads, item_cap=max(n_est, 1))
    got_st = dec["status"][:nb].cpu().numpy()
    assert np.array_equal(got_st, status), "decode statuses differ from the oracle"
    if expect_status_ok:
        assert (status == 0).all(), "oracle rejects a block"
    assert np.array_equal(dec["item_start"][:nb + 1].cpu().numpy().view(np.uint32), item_start), "item_start"
    n = int(item_start[-1])
    for f in fields:
        g = dec[f][:n].cpu().numpy().view(FIELD_NP[f])
        assert np.array_equal(g, parsed[f].astype(FIELD_NP[f])), f"decoded field {f} differs from the oracle"
    return n


# ------------------------------------------------------------- CPU baseline
def cpu_info():
    """Host CPUs as the process sees them: nproc-style affinity count, the
    machine's CPU count, and the cgroup CPU quota if one is set."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    return {"nproc": aff, "cpu_count": os.cpu_count(), "cgroup_cpu_quota": quota, "cpu_model": cpu_model()}


def cpu_baseline(ref_buf, ref_off, items_host, starts_np, sample_blocks=300000, min_seconds=2.0, world=1):
    """The oracle (C restatement of the reference path, AVX2 XXH3) on the host
    cores, same workload: encode (DataBlock::encode_into + Block::write_into) and
    decode (Block::from_file + DataBlock::iter into the same parsed SoA as the
    GPU) of a bounded sample of the batch (300 K blocks, 1.1 GB: larger than the
    host's L3); 1 thread, the per-GPU CPU share (16) and every core available to
    the process (affinity mask capped by the cgroup quota / the box's per-GPU
    share).  `value` is the all-available-cores figure."""
    import numpy as np
    import pyoracle
    nb = min(sample_blocks, len(ref_off) - 1)
    n_items = int(starts_np[nb])
    off = np.ascontiguousarray(ref_off[:nb + 1])
    blocks = ref_buf[:int(off[-1])]
    nbytes = int(off[-1])
    ko = items_host.key_off[:n_items + 1]
    vo = items_host.val_off[:n_items + 1]
    it = pyoracle.Items(items_host.keys[:int(ko[-1])], ko, items_host.vals[:int(vo[-1])], vo,
                        items_host.seqno[:n_items], items_host.vtype[:n_items])
    st = np.ascontiguousarray(starts_np[:nb + 1], np.uint32)

    def rate(fn, threads):
        passes, t0 = 0, time.perf_counter()
        while True:
            fn(threads)
            passes += 1
            el = time.perf_counter() - t0
            if el >= min_seconds or passes >= 200:
                return nbytes * passes / el / 2 ** 30

    def enc(t):
        b, o = pyoracle.encode_blocks(it, st, nthreads=t)
        assert int(o[-1]) == nbytes

    def dec(t):
        _, _, s = pyoracle.decode_blocks(blocks, off, nthreads=t, item_cap=n_items)
        assert (s == 0).all()

    info = cpu_info()
    share = max(1, min(HOST_THREADS, info["nproc"] // max(1, world)))
    # every core this process may use: the affinity mask, capped by the cgroup CPU quota (on the GPU
    # box the harness gives one GPU a 16-CPU share of a larger machine; more threads would only
    # time-slice on that share and break its worker-pool rule)
    avail = info["nproc"] if info["cgroup_cpu_quota"] is None else min(info["nproc"], int(info["cgroup_cpu_quota"]))
    if os.environ.get("GRAFT_REPO_ROOT"):  # (the GPU box: its per-GPU CPU share)
        avail = min(avail, HOST_THREADS)
    tall = max(1, avail // max(1, world))
    res = {}
    for t in sorted({1, share, tall}):
        e, d = rate(enc, t), rate(dec, t)
        res[t] = {"encode_GiB_per_s": round(e, 3), "decode_GiB_per_s": round(d, 3),
                  "round_trip_GiB_per_s": round(1.0 / (1.0 / e + 1.0 / d), 3)}
    return {"value": res[tall]["round_trip_GiB_per_s"], "unit": "GiB/s", "cores": tall, "kind": "port",
            **info, "per_gpu_share_threads": share, "threads": {str(k): v for k, v in res.items()},
            "sample": f"{nb} blocks ({nbytes / 1e9:.2f} GB, > L3) of the same batch, encode then decode, each leg "
                      f"repeated >= {min_seconds:.0f} s; value = block bytes / (t_enc + t_dec) with {tall} threads "
                      f"(every core available to the process: affinity {info['nproc']}, cgroup quota "
                      f"{info['cgroup_cpu_quota']}; 1 and {share} threads alongside) "
                      f"(oracle/batch.c, AVX2 XXH3, -O3 -march=x86-64-v3)"}


# ----------------------------------------------------------------- ceilings
def ceilings(torch, nbytes=4 << 30, reps=5):
    """Practical HBM ceilings measured in this run (lsm-tree_amd/ceiling):
    a 16 B/lane streaming copy (R+W) and the decode kernel's LDS-DMA read shape."""
    lib = C.CDLL(str(ROOT / "lsm-tree_amd" / "ceiling" / "liblsmceiling.so"))
    lib.lsm_ceiling_copy.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p]
    lib.lsm_ceiling_read.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p]
    src = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    src.random_(0, 256)
    dst = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    sink = torch.zeros(4, dtype=torch.int32, device="cuda")
    s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    out = {}
    for name, fn, moved in (("copy", lambda: lib.lsm_ceiling_copy(src.data_ptr(), dst.data_ptr(), nbytes, s),
                             2 * nbytes),
                            ("read", lambda: lib.lsm_ceiling_read(src.data_ptr(), nbytes, sink.data_ptr(), s),
                             nbytes)):
        assert fn() == 0
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        out[f"{name}_GBps"] = round(moved / (ms * 1e-3) / 1e9, 1)
    del src, dst
    torch.cuda.empty_cache()
    return out


# ------------------------------------------------------------- side legs
def time_decode(torch, lsmgpu, blocks, boff, nb, n_items, steps, fields=DATA_FIELDS):
    """Device-resident lsm_decode_blocks over a batch (count + scan + verify +
    parse), HIP events on the launch stream; checks every status and the count."""
    dec = lsmgpu.Decoder(blocks.device)
    out = dec.alloc_outputs(n_items, nb, fields=fields)
    dec.decode(blocks, boff, nb, out, n_items)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(steps):
        dec.decode(blocks, boff, nb, out, n_items)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / steps, out


def bench_config4(torch, lsmgpu, steps, rank, threads):
    """configs[3]: prefix-heavy keys (32 B shared prefix + 8 B suffix), 256 B
    values, 16 KiB blocks (56 items, 14953 B on disk), 262144 blocks; every
    block checked against the oracle (encode bytes and decoded fields)."""
    nb = 262144
    check_cut_rule(lsmgpu, 56, 40, 256, 16384)
    items, starts, n = make_workload(torch, lsmgpu, nb, items_per_block=56, key_len=40, val_len=256,
                                     seed=0x5EED0004 + rank, kind="prefix")
    enc_ctx = lsmgpu.Encoder()
    enc = enc_ctx.encode(items, starts, nb)
    torch.cuda.synchronize()
    total = int(enc["block_off"][nb].item())
    assert int(enc["block_off"][1].item()) == 14953  # SURVEY 8 table (first block; later ones vary by a byte)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(3):
        enc_ctx.encode(items, starts, nb, out=enc)
    e1.record()
    torch.cuda.synchronize()
    enc_ms = e0.elapsed_time(e1) / 3
    dec_ms, out = time_decode(torch, lsmgpu, enc["buf"], enc["block_off"], nb, n, steps)
    ref_buf, ref_off = check_encode_all(torch, items, starts, enc, nb, n, threads)
    check_decode_all(out, ref_buf, ref_off, nb, threads)
    res = {"workload": "BASELINE configs[3]: 16 KiB blocks, 32 B shared prefix + 8 B suffix keys, 256 B values",
           "blocks": nb, "bytes": total, "decode_ms": round(dec_ms, 4),
           "decode_GiB_per_s": round(total / (dec_ms * 1e-3) / 2 ** 30, 3),
           "encode_ms": round(enc_ms, 4), "encode_GiB_per_s": round(total / (enc_ms * 1e-3) / 2 ** 30, 3),
           "round_trip_GiB_per_s": round(total / ((enc_ms + dec_ms) * 1e-3) / 2 ** 30, 3),
           "oracle_checked_blocks": nb}
    del items, enc, out, ref_buf
    torch.cuda.empty_cache()
    return res


# configs[4] mix: equal bytes of 4/16/64 KiB data blocks with counter (G1)
# and random sorted (G2) 16 B keys / 64 B values, plus one full index block
# (RI 1) per 64 MiB "table" (flush target, src/tree/mod.rs:374-377).
C5_SEGMENTS = [(4096, 52, "counter", 3769), (4096, 52, "random", 4466), (16384, 205, "counter", 14636),
               (16384, 205, "random", 17300), (65536, 820, "counter", 58309), (65536, 820, "random", 69219)]
C5_TABLE = 64 << 20


def build_config5_shard(torch, lsmgpu, shard_bytes, rank, threads):
    """This rank's byte share of the configs[4] batch, GPU-encoded: data blocks
    of the six segments, each followed by its index blocks (one per table).
    Every data and index block's bytes are checked against the oracle."""
    import numpy as np
    segs, n_items, n_data_blocks, n_index_blocks = [], 0, 0, 0
    checked = 0
    for si, (bs, ipb, kind, est) in enumerate(C5_SEGMENTS):
        nb = max(1, int(shard_bytes / len(C5_SEGMENTS) / est))
        check_cut_rule(lsmgpu, ipb, 16, 64, bs)
        items, starts, n = make_workload(torch, lsmgpu, nb, items_per_block=ipb, seed=0x5EED0005 + 97 * rank + si,
                                         kind=kind)
        enc = lsmgpu.Encoder().encode(items, starts, nb)
        torch.cuda.synchronize()
        check_encode_all(torch, items, starts, enc, nb, n, threads)
        boff = enc["block_off"][:nb + 1]
        dev = boff.device
        # index entries: end key, seqno of each block's last item, handle (offset in its table, size)
        last = starts[1:].to(torch.int64) - 1
        end_keys = items["keys"][:n * 16].view(n, 16)[last].reshape(-1)
        table = torch.div(boff[:-1], C5_TABLE, rounding_mode="floor")
        tfirst = torch.ones(nb, dtype=torch.bool, device=dev)
        tfirst[1:] = table[1:] != table[:-1]
        first = torch.nonzero(tfirst).flatten()
        tid = torch.cumsum(tfirst.to(torch.int64), 0) - 1
        ix = {"keys": torch.cat([end_keys, torch.zeros(lsmgpu.LSM_INPUT_PADDING, dtype=torch.uint8, device=dev)]),
              "key_off": torch.arange(nb + 1, dtype=torch.int64, device=dev) * 16,
              "seqno": items["seqno"][last].contiguous(),
              "handle_off": (boff[:-1] - boff[first][tid]).contiguous(),
              "handle_size": (boff[1:] - boff[:-1]).to(torch.int32).contiguous()}
        istarts = torch.cat([first, torch.tensor([nb], device=dev)]).to(torch.int32)
        nt = int(first.numel())
        ienc = lsmgpu.Encoder().encode(ix, istarts, nt, restart_interval=1, block_type=lsmgpu.BLOCK_INDEX)
        torch.cuda.synchronize()
        check_encode_all(torch, ix, istarts, ienc, nt, nb, threads, restart_interval=1, block_type=1)
        checked += nb + nt
        dbytes, ibytes = int(boff[nb].item()), int(ienc["block_off"][nt].item())
        segs.append((enc["buf"][:dbytes], boff[:-1].clone(), ienc["buf"][:ibytes], ienc["block_off"][:nt] + dbytes,
                     dbytes + ibytes))
        n_items += n + nb
        n_data_blocks += nb
        n_index_blocks += nt
        del items, enc, ienc, ix
    base, pieces, offl = 0, [], []
    for dbuf, doff, ibuf, ioff, seg_bytes in segs:
        pieces += [dbuf, ibuf]
        offl += [doff + base, ioff + base]
        base += seg_bytes
    pieces.append(torch.zeros(lsmgpu.LSM_INPUT_PADDING, dtype=torch.uint8, device=pieces[0].device))
    blocks = torch.cat(pieces)
    block_off = torch.cat(offl + [torch.tensor([base], dtype=torch.int64, device=blocks.device)])
    del segs, pieces
    torch.cuda.empty_cache()
    return blocks, block_off, n_data_blocks + n_index_blocks, n_items, base, n_index_blocks, checked


def bench_config5(torch, lsmgpu, steps, rank, world, dist, dev, threads, total_bytes=8 << 30):
    """configs[4]: 8 GiB of mixed data + index blocks, byte-split across the
    ranks (strong scaling: the batch is fixed, each rank decodes its share).
    Every block's decode (status, item_start, all fields incl. handle_off) is
    checked against the oracle."""
    import numpy as np
    blocks, boff, nb, n_items, nbytes, n_idx, checked = build_config5_shard(torch, lsmgpu, total_bytes / world,
                                                                            rank, threads)
    ms, out = time_decode(torch, lsmgpu, blocks, boff, nb, n_items, steps, fields=DATA_FIELDS + ["handle_off"])
    host = blocks[:nbytes].cpu().numpy()
    hoff = boff.cpu().numpy().view(np.uint64)
    check_decode_all(out, host, hoff, nb, threads, fields=DATA_FIELDS + ["handle_off"])
    del host
    t = torch.tensor([ms, float(nbytes)], dtype=torch.float64, device=dev)
    if dist is not None:
        mx = t.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        sm = t.clone()
        dist.all_reduce(sm, op=dist.ReduceOp.SUM)
        ms_all, bytes_all = float(mx[0].item()), float(sm[1].item())
    else:
        ms_all, bytes_all = ms, float(nbytes)
    del blocks, boff, out
    torch.cuda.empty_cache()
    return {"workload": "BASELINE configs[4]: 8 GiB mixed 4/16/64 KiB data (G1+G2 keys) + index blocks, "
                        "byte-split across ranks (strong scaling)",
            "total_bytes": int(bytes_all), "blocks_per_rank": nb, "index_blocks_per_rank": n_idx,
            "decode_ms_max_rank": round(ms_all, 4), "GiB_per_s": round(bytes_all / (ms_all * 1e-3) / 2 ** 30, 3),
            "oracle_checked_blocks_per_rank": {"encode": checked, "decode": nb}}


def bench_large_blocks(torch, lsmgpu, threads, steps=5):
    """Data blocks above the general path's 72 KiB stage (the writer's data_block_size
    goes up to 4 MiB, writer/mod.rs:193-198): 240 x 1 MiB and 60 x 4 MiB blocks of
    16 B counter keys / 64 B values, encoded and decoded across the whole GPU (the
    wrappers hand the workspace pool for batches of such blocks); every block
    checked against the oracle (encoded bytes and decoded fields)."""
    res = {}
    for name, nb, ipb, bs in (("1MiB", 240, 13108, 1 << 20), ("4MiB", 60, 52429, 4 << 20)):
        check_cut_rule(lsmgpu, ipb, 16, 64, bs)  # = the writer's cut at that data_block_size
        items, starts, n = make_workload(torch, lsmgpu, nb, items_per_block=ipb, seed=0x5EED0007)
        enc_ctx = lsmgpu.Encoder()
        enc = enc_ctx.encode(items, starts, nb)
        torch.cuda.synchronize()
        total = int(enc["block_off"][nb].item())
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(3):
            enc_ctx.encode(items, starts, nb, out=enc)
        e1.record()
        torch.cuda.synchronize()
        enc_ms = e0.elapsed_time(e1) / 3
        dec_ms, out = time_decode(torch, lsmgpu, enc["buf"], enc["block_off"], nb, n, steps)
        ref_buf, ref_off = check_encode_all(torch, items, starts, enc, nb, n, threads)
        check_decode_all(out, ref_buf, ref_off, nb, threads)
        res[name] = {"blocks": nb, "bytes": total, "encode_ms": round(enc_ms, 3),
                     "encode_GiB_per_s": round(total / (enc_ms * 1e-3) / 2 ** 30, 2), "decode_ms": round(dec_ms, 3),
                     "decode_GiB_per_s": round(total / (dec_ms * 1e-3) / 2 ** 30, 2), "oracle_checked_blocks": nb}
        del items, enc, out, ref_buf
        torch.cuda.empty_cache()
    res["note"] = ("the workspace pool (lsm_*_workspace_size_ex) spreads each block over the GPU: encode = "
                   "item-parallel plan (E1p), record units assembled in LDS (their KiB contributions from the "
                   "image) + 16-B copy-out, the leftover KiB blocks, one wave per block for the eight XXH3 "
                   "chains + header; decode = unit table, 32 KiB staged windows (phase A on one wave while three "
                   "reduce KiB contributions; interval walks for odd shapes), one wave per block for the chains "
                   "+ checksum + status")
    return res


def bench_hash_index(torch, lsmgpu, steps, threads, nb=1 << 20, ratio=1.33, n_queries=1 << 20, reps=5):
    """The configs[1] batch with the data-block hash index (data_block_hash_ratio
    1.33, src/config/mod.rs:286, hash_index/builder.rs:64-110): encode (the
    bucket votes in encode_group_kernel<*, true>), decode, and point reads that
    take the hash probe first.  Every block checked against the oracle."""
    items, starts, n = make_workload(torch, lsmgpu, nb, seed=0x5EED0008)
    enc_ctx = lsmgpu.Encoder()
    enc = enc_ctx.encode(items, starts, nb, hash_ratio=ratio)
    torch.cuda.synchronize()
    total = int(enc["block_off"][nb].item())
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(steps):
        enc_ctx.encode(items, starts, nb, hash_ratio=ratio, out=enc)
    e1.record()
    torch.cuda.synchronize()
    enc_ms = e0.elapsed_time(e1) / steps
    dec_ms, out = time_decode(torch, lsmgpu, enc["buf"], enc["block_off"], nb, n, steps)
    ref_buf, ref_off = check_encode_all(torch, items, starts, enc, nb, n, threads, hash_ratio=ratio)
    check_decode_all(out, ref_buf, ref_off, nb, threads)
    del out, ref_buf
    g = torch.Generator(device="cuda")
    g.manual_seed(0x5EED0009)
    qi = torch.randint(0, n, (n_queries,), dtype=torch.int64, device="cuda", generator=g)
    qb = torch.div(qi, 52, rounding_mode="floor").to(torch.int32)
    needles = torch.cat([items["keys"][:n * 16].view(n, 16)[qi].reshape(-1),
                         torch.zeros(lsmgpu.LSM_INPUT_PADDING, dtype=torch.uint8, device="cuda")])
    noff = torch.arange(n_queries + 1, dtype=torch.int64, device="cuda") * 16
    snap = torch.full((n_queries,), (1 << 63) - 1, dtype=torch.int64, device="cuda")
    pr = lsmgpu.point_read(enc["buf"], enc["block_off"], nb, qb, needles, noff, snap)
    torch.cuda.synchronize()
    assert int((pr["status"] != 0).sum().item()) == 0
    assert bool((pr["item"].to(torch.int64) == qi - qb.to(torch.int64) * 52).all().item()), "point_read hits"
    e0.record()
    for _ in range(reps):
        lsmgpu.point_read(enc["buf"], enc["block_off"], nb, qb, needles, noff, snap)
    e1.record()
    torch.cuda.synchronize()
    pr_ms = e0.elapsed_time(e1) / reps
    res = {"workload": f"configs[1] shape (1 M x 4 KiB, 16 B keys, 64 B values) with hash ratio {ratio}",
           "blocks": nb, "bytes": total, "encode_ms": round(enc_ms, 4),
           "encode_GiB_per_s": round(total / (enc_ms * 1e-3) / 2 ** 30, 3), "decode_ms": round(dec_ms, 4),
           "decode_GiB_per_s": round(total / (dec_ms * 1e-3) / 2 ** 30, 3),
           "point_read_ms": round(pr_ms, 4), "point_read_Mqueries_per_s": round(n_queries / pr_ms / 1e3, 1),
           "oracle_checked_blocks": nb}
    del items, enc
    torch.cuda.empty_cache()
    return res


def bench_point_read(torch, lsmgpu, items, enc, nb, n_items, n_queries=1 << 20, reps=5):
    """Batched DataBlock::point_read: random existing keys of the config 2 batch,
    snapshot = max; every query must hit its own item."""
    g = torch.Generator(device="cuda")
    g.manual_seed(0x5EED0006)
    qi = torch.randint(0, n_items, (n_queries,), dtype=torch.int64, device="cuda", generator=g)
    qb = torch.div(qi, 52, rounding_mode="floor").to(torch.int32)
    needles = torch.cat([items["keys"][:n_items * 16].view(n_items, 16)[qi].reshape(-1),
                         torch.zeros(lsmgpu.LSM_INPUT_PADDING, dtype=torch.uint8, device="cuda")])
    noff = torch.arange(n_queries + 1, dtype=torch.int64, device="cuda") * 16
    snap = torch.full((n_queries,), (1 << 63) - 1, dtype=torch.int64, device="cuda")
    out = lsmgpu.point_read(enc["buf"], enc["block_off"], nb, qb, needles, noff, snap)
    torch.cuda.synchronize()
    assert int((out["status"] != 0).sum().item()) == 0
    assert bool((out["item"].to(torch.int64) == qi - qb.to(torch.int64) * 52).all().item()), "point_read hits"
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        lsmgpu.point_read(enc["buf"], enc["block_off"], nb, qb, needles, noff, snap)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    # range seeks: [key(i), key(i + 20)] inside the block of i (Table::range's per-block step)
    lo_i = qi
    hi_i = torch.minimum(qi + 20, (qb.to(torch.int64) + 1) * 52 - 1)
    kv = items["keys"][:n_items * 16].view(n_items, 16)
    pad = torch.zeros(lsmgpu.LSM_INPUT_PADDING, dtype=torch.uint8, device="cuda")
    lo = torch.cat([kv[lo_i].reshape(-1), pad])
    hi = torch.cat([kv[hi_i].reshape(-1), pad])
    flags = torch.full((n_queries,), lsmgpu.SEEK_LO | lsmgpu.SEEK_HI, dtype=torch.uint8, device="cuda")
    sk = lsmgpu.seek(enc["buf"], enc["block_off"], nb, qb, lo, noff, hi, noff, flags)
    torch.cuda.synchronize()
    base = qb.to(torch.int64) * 52
    assert int((sk["status"] != 0).sum().item()) == 0
    assert bool((sk["first"].to(torch.int64) == lo_i - base).all().item()), "seek lower bounds"
    assert bool((sk["end"].to(torch.int64) == hi_i - base + 1).all().item()), "seek upper bounds"
    e0.record()
    for _ in range(reps):
        lsmgpu.seek(enc["buf"], enc["block_off"], nb, qb, lo, noff, hi, noff, flags)
    e1.record()
    torch.cuda.synchronize()
    ms_seek = e0.elapsed_time(e1) / reps
    return {"queries": n_queries, "ms": round(ms, 4), "Mqueries_per_s": round(n_queries / ms / 1e3, 1),
            "seek_ms": round(ms_seek, 4), "seek_Mqueries_per_s": round(n_queries / ms_seek / 1e3, 1),
            "note": "lane per query straight from HBM (restart binary search + MVCC scan); seek = lower + upper "
                    "bound of a 21-key range per query"}


def bench_file_checksum(torch, lsmgpu, enc, total_bytes, reps=5):
    """Whole-file xxh3_128 (ChecksummedWriter digest, src/checksum.rs:59-96) over
    the encoded configs[1] batch taken as one file."""
    lsmgpu.xxh3_128_file(enc["buf"], total_bytes)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        lsmgpu.xxh3_128_file(enc["buf"], total_bytes)  # (returns the digest: synchronises)
    ms = (time.perf_counter() - t0) * 1e3 / reps
    return {"bytes": total_bytes, "ms": round(ms, 4), "GiB_per_s": round(total_bytes / (ms * 1e-3) / 2 ** 30, 1),
            "note": "per-KiB XXH3 contributions across the GPU, then one wave's scramble chain; "
                    "host-timed incl. the 16-B digest copy"}


def bench_file_checksum_batch(torch, lsmgpu, enc, total_bytes, n_files=64, reps=5):
    """Running whole-file checksums of n_files tables advanced together
    (lsm_xxh3_128_stream_update_batch: one ChecksummedWriter per table of a
    MultiWriter, src/table/multi_writer.rs:181-257): the encoded configs[1] batch
    cut into n_files equal files (~62 MB each), every digest checked against the
    oracle's one-shot xxh3_128 outside the timed region."""
    import numpy as np
    import pyoracle
    per = total_bytes // n_files
    off = torch.arange(n_files + 1, dtype=torch.int64, device=enc["buf"].device) * per
    w = lsmgpu.ChecksummedWriterSet(n_files)
    st = w.write(enc["buf"], off, per * n_files)
    got = w.checksums()
    assert int((st[:n_files] != 0).sum()) == 0
    host = enc["buf"][:per * n_files].cpu().numpy()
    for i in range(n_files):
        exp = pyoracle.xxh3_128(host[i * per:(i + 1) * per].tobytes())
        assert (got[i][1] << 64) | got[i][0] == exp, f"batched checksum of file {i} differs from the oracle"
    del host
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        ws = lsmgpu.ChecksummedWriterSet(n_files)
        ws.write(enc["buf"], off, per * n_files)
        ws.checksums()  # (synchronises)
    ms = (time.perf_counter() - t0) * 1e3 / reps
    nbytes = per * n_files
    return {"files": n_files, "bytes_per_file": per, "ms": round(ms, 4),
            "GiB_per_s": round(nbytes / (ms * 1e-3) / 2 ** 30, 1),
            "note": "init + one update_batch + digest_batch per rep, host-timed incl. the digest copy; "
                    "every digest equals the oracle's one-shot xxh3_128"}


def bench_bloom(torch, lsmgpu, items, n_items, reps=5):
    """Standard Bloom filter over the configs[1] batch's keys (FullFilterWriter,
    src/table/writer/filter/full.rs:47-92, BitsPerKey(10) default)."""
    out = {}
    for name, n in (("table_1M", min(1 << 20, n_items)), ("batch", n_items)):
        ko = items["key_off"][:n + 1]
        m, k = lsmgpu.bloom_shape(n, bpk=10.0)
        h = lsmgpu.hash64_keys(items["keys"], ko)
        filt = lsmgpu.bloom_build(h, m, k)
        hit = lsmgpu.bloom_contains(filt, h)
        torch.cuda.synchronize()
        assert int((hit != 1).sum().item()) == 0, "bloom: false negative"
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        ev[0].record()
        for _ in range(reps):
            h = lsmgpu.hash64_keys(items["keys"], ko)
        ev[1].record()
        for _ in range(reps):
            filt = lsmgpu.bloom_build(h, m, k)
        ev[2].record()
        for _ in range(reps):
            hit = lsmgpu.bloom_contains(filt, h)
        ev[3].record()
        torch.cuda.synchronize()
        t = [ev[i].elapsed_time(ev[i + 1]) / reps for i in range(3)]
        out[name] = {"keys": n, "m_bits": m, "k": k, "hash64_ms": round(t[0], 4), "build_ms": round(t[1], 4),
                     "probe_ms": round(t[2], 4), "Mkeys_per_s_build": round(n / (t[0] + t[1]) / 1e3, 1),
                     "Mprobes_per_s": round(n / t[2] / 1e3, 1)}
    return out


def bench_lz4(torch, lsmgpu, enc, n_blocks, reps=5, sample=131072):
    """Block::from_reader with CompressionType::Lz4 (src/table/block/mod.rs:87-128)
    over LZ4 copies of the first `sample` configs[1] blocks (payloads compressed on
    the host by liblz4, pyarrow "lz4_raw", headers sealed with python-xxhash),
    checked + decompressed on the device."""
    import numpy as np
    try:
        import pyarrow as pa
        import xxhash
    except ImportError as e:
        return {"skipped": str(e)}
    nb = min(sample, n_blocks)
    off = enc["block_off"][:nb + 1].cpu().numpy().astype(np.int64)
    host = enc["buf"][:int(off[-1])].cpu().numpy().tobytes()
    codec = pa.Codec("lz4_raw")
    parts, raw_total = [], 0
    for b in range(nb):
        payload = host[off[b] + 33:off[b + 1]]
        c = codec.compress(payload, asbytes=True)
        h = b"LSM\x03\x00" + xxhash.xxh3_128_intdigest(c).to_bytes(16, "little") + len(c).to_bytes(4, "little") + \
            len(payload).to_bytes(4, "little")
        parts.append(h + xxhash.xxh3_128_intdigest(h).to_bytes(16, "little")[:4] + c)
        raw_total += len(payload)
    loff = np.zeros(nb + 1, np.int64)
    loff[1:] = np.cumsum([len(p) for p in parts])
    dbuf = lsmgpu.to_device_bytes(np.frombuffer(b"".join(parts), np.uint8))
    doff = torch.from_numpy(loff).cuda()
    out, out_off, status = lsmgpu.lz4_decompress_blocks(dbuf, doff)
    torch.cuda.synchronize()
    assert int((status != 0).sum().item()) == 0, "lz4: block status"
    raw = b"".join(host[off[b] + 33:off[b + 1]] for b in range(nb))
    assert out[:len(raw)].cpu().numpy().tobytes() == raw, "lz4: decompressed bytes"
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        lsmgpu.lz4_decompress_blocks(dbuf, doff)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    # LZ4 -> parse chain (Block::from_reader(Lz4) + DataBlock::iter): every field vs the plain decode
    ch = lsmgpu.decode_lz4_blocks(dbuf, doff, expect_type=0, item_cap=nb * 52, fields=DATA_FIELDS)
    torch.cuda.synchronize()
    assert int((ch["status"][:nb] != 0).sum().item()) == 0, "lz4 chain: status"
    ref = lsmgpu.decode_blocks(enc["buf"], enc["block_off"][:nb + 1], nb, item_cap=nb * 52, fields=DATA_FIELDS)
    torch.cuda.synchronize()
    for f in DATA_FIELDS:
        assert torch.equal(ch[f][:nb * 52], ref[f][:nb * 52]), f"lz4 chain: {f}"
    del ch, ref
    t0 = time.perf_counter()
    for _ in range(reps):
        lsmgpu.decode_lz4_blocks(dbuf, doff, expect_type=0, item_cap=nb * 52, fields=DATA_FIELDS)
    torch.cuda.synchronize()
    ms_chain = (time.perf_counter() - t0) * 1e3 / reps
    # the same chain without the host sync: the frame arena sized by the caller (raw bytes
    # + one 33-B frame header per block: what the plan would find), lsm_lz4_plan_capped
    fcap = raw_total + 33 * nb
    ch = lsmgpu.decode_lz4_blocks(dbuf, doff, expect_type=0, item_cap=nb * 52, fields=DATA_FIELDS, frames_cap=fcap)
    torch.cuda.synchronize()
    assert int((ch["status"][:nb] != 0).sum().item()) == 0, "lz4 capped chain: status"
    del ch
    t0 = time.perf_counter()
    for _ in range(reps):
        lsmgpu.decode_lz4_blocks(dbuf, doff, expect_type=0, item_cap=nb * 52, fields=DATA_FIELDS, frames_cap=fcap)
    torch.cuda.synchronize()
    ms_capped = (time.perf_counter() - t0) * 1e3 / reps
    return {"blocks": nb, "stored_bytes": int(loff[-1]), "raw_bytes": raw_total, "ms": round(ms, 4),
            "chain_capped_ms": round(ms_capped, 4),
            "chain_capped_GiB_per_s_raw": round(raw_total / (ms_capped * 1e-3) / 2 ** 30, 1),
            "GiB_per_s_raw": round(raw_total / (ms * 1e-3) / 2 ** 30, 1),
            "note": "plan (verified headers -> output offsets) + header / xxh3_128 verify + LZ4 decode, every "
                    "decompressed byte checked",
            "chain_ms": round(ms_chain, 4), "chain_GiB_per_s_raw": round(raw_total / (ms_chain * 1e-3) / 2 ** 30, 1),
            "chain_note": "decode_lz4_blocks: plan_framed (host sync for the arena size) + decompress_framed + "
                          "decode with LSM_DECODE_PAYLOAD_VERIFIED, host-timed; every parsed field equal to the "
                          "plain decode of the uncompressed blocks"}


def bench_table_scan(torch, lsmgpu, items, enc, nb, n_items, ref_out, reps=3, partition=100):
    """Scanner over one table whose data region is the whole configs[1] batch
    (scanner.rs:24-92): a two-level block index is written on the
    device with lsm_encode_blocks(block_type = Index) (KeyedBlockHandle(last key,
    seqno, (offset, size)) per data block, partitions of `partition` handles, a TLI
    of partition handles, writer/index/partitioned.rs), appended after the data;
    lsm_scan_table then decodes TLI -> partitions -> every data block
    (global_seqno 1000 added).  Checked: block offsets, statuses and every item's
    fields equal the plain decode's (seqno + 1000)."""
    dev = enc["buf"].device
    data_len = int(enc["block_off"][nb].item())
    boff = enc["block_off"][:nb + 1]
    last = (torch.arange(1, nb + 1, device=dev, dtype=torch.int64) * 52 - 1)
    kl = 16

    def index_blocks(end_items_key, seq, h_off, h_size, per_block, base):
        n = h_off.numel()
        nblk = (n + per_block - 1) // per_block
        it = {"keys": end_items_key, "key_off": torch.arange(n + 1, device=dev, dtype=torch.int64) * kl,
              "seqno": seq, "handle_off": h_off, "handle_size": h_size.to(torch.int32)}
        st = torch.clamp(torch.arange(nblk + 1, device=dev, dtype=torch.int64) * per_block, max=n).to(torch.int32)
        out = lsmgpu.Encoder(dev).encode(it, st, nblk, block_type=lsmgpu.BLOCK_INDEX)
        torch.cuda.synchronize()
        assert int((out["status"][:nblk] != 0).sum().item()) == 0
        ln = int(out["block_off"][nblk].item())
        return out["buf"][:ln], out["block_off"][:nblk + 1] + base, nblk

    ekeys = items["keys"][:n_items * kl].view(n_items, kl)[last].reshape(-1)
    ekeys = torch.cat([ekeys, torch.zeros(64, dtype=torch.uint8, device=dev)])
    seq = items["seqno"][last]
    parts, poff, npart = index_blocks(ekeys, seq, boff[:nb], (boff[1:] - boff[:nb]), partition, data_len)
    plast = torch.clamp(torch.arange(1, npart + 1, device=dev) * partition, max=nb) - 1
    pkeys = torch.cat([ekeys[:nb * kl].view(nb, kl)[plast].reshape(-1), torch.zeros(64, dtype=torch.uint8, device=dev)])
    tli, toff, _ = index_blocks(pkeys, seq[plast], poff[:npart], poff[1:] - poff[:npart], 1 << 20,
                                data_len + parts.numel())
    file_len = data_len + parts.numel() + tli.numel()
    f = lsmgpu.padded_bytes(file_len, dev)
    f[:data_len].copy_(enc["buf"][:data_len])
    f[data_len:data_len + parts.numel()].copy_(parts)
    f[data_len + parts.numel():file_len].copy_(tli)
    tli_off = data_len + parts.numel()
    kw = dict(two_level=True, global_seqno=1000, block_count=nb, cap_blocks=nb + 16, item_cap=n_items,
              fields=DATA_FIELDS)
    out = lsmgpu.scan_table(f, file_len, tli_off, tli.numel(), **kw)
    torch.cuda.synchronize()
    assert out["table_status"] == 0 and out["n_blocks"] == nb, (out["table_status"], out["n_blocks"])
    assert torch.equal(out["block_off"], boff)
    assert int((out["status"][:nb] != 0).sum().item()) == 0
    assert torch.equal(out["seqno"][:n_items], ref_out["seqno"][:n_items] + 1000)
    for fld in DATA_FIELDS[1:]:
        assert torch.equal(out[fld][:n_items], ref_out[fld][:n_items]), fld
    del out
    t0 = time.perf_counter()
    for _ in range(reps):
        lsmgpu.scan_table(f, file_len, tli_off, tli.numel(), **kw)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / reps
    # without host synchronisation: lsm_scan_table_async, bounds from the metadata's block
    # count and the TLI size (at most one partition handle per 4 TLI bytes)
    kwa = dict(kw, sync=False, data_blocks_hint=nb, index_blocks_hint=int(tli.numel()) // 4)
    outa = lsmgpu.scan_table(f, file_len, tli_off, tli.numel(), **kwa)
    torch.cuda.synchronize()
    assert int(outa["table_status"].item()) == 0 and int(outa["n_blocks"].item()) == nb
    assert torch.equal(outa["block_off"][:nb + 1], boff) and int((outa["status"][:nb] != 0).sum().item()) == 0
    assert torch.equal(outa["seqno"][:n_items], ref_out["seqno"][:n_items] + 1000)
    for fld in DATA_FIELDS[1:]:
        assert torch.equal(outa[fld][:n_items], ref_out[fld][:n_items]), fld
    del outa
    t0 = time.perf_counter()
    for _ in range(reps):
        lsmgpu.scan_table(f, file_len, tli_off, tli.numel(), **kwa)
    torch.cuda.synchronize()
    ms_a = (time.perf_counter() - t0) * 1e3 / reps
    return {"data_blocks": nb, "index_partitions": npart, "tli_bytes": int(tli.numel()), "file_bytes": file_len,
            "ms": round(ms, 4), "GiB_per_s": round(file_len / (ms * 1e-3) / 2 ** 30, 1),
            "async_ms": round(ms_a, 4), "async_GiB_per_s": round(file_len / (ms_a * 1e-3) / 2 ** 30, 1),
            "note": "host-timed lsm_scan_table call (2 index levels, one stream sync each, then the data decode); "
                    "async: lsm_scan_table_async (no host sync; partitions bounded by tli_size / 4, data blocks by "
                    "the block count); every item equal to the plain decode with global_seqno 1000 added"}


def bench_materialize(torch, lsmgpu, enc, nb, out, n_items, reps=5):
    """DataBlockParsedItem::materialize on the device (data_block/mod.rs:296-315) for
    every item of the configs[1] decode: keys = restart-head prefix || suffix; checked
    against the encoder's input keys."""
    keys, key_off = lsmgpu.materialize_keys(enc["buf"], enc["block_off"], nb, out, n_items)
    torch.cuda.synchronize()
    total = int(key_off[n_items].item())
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        lsmgpu.materialize_keys(enc["buf"], enc["block_off"], nb, out, n_items)
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / reps
    # the sync-free form: an arena the caller sized (here: exactly), lsm_materialize_keys_capped
    k2, o2, res = lsmgpu.materialize_keys(enc["buf"], enc["block_off"], nb, out, n_items, key_cap=total)
    torch.cuda.synchronize()
    assert int(res.item()) == 0 and torch.equal(o2, key_off) and torch.equal(k2[:total], keys[:total])
    del k2
    a.record()
    for _ in range(reps):
        lsmgpu.materialize_keys(enc["buf"], enc["block_off"], nb, out, n_items, key_cap=total)
    b.record()
    torch.cuda.synchronize()
    ms_c = a.elapsed_time(b) / reps
    return keys[:total], {"items": n_items, "key_bytes": total, "ms": round(ms, 4),
                          "GiB_per_s_keys": round(total / (ms * 1e-3) / 2 ** 30, 1),
                          "capped_ms": round(ms_c, 4), "capped_GiB_per_s_keys": round(total / (ms_c * 1e-3) / 2 ** 30, 1),
                          "note": "plan (lengths + scan) + copy, host-synchronised once for the arena size; capped: "
                                  "lsm_materialize_keys_capped into an arena sized by the caller, no host sync, "
                                  "same keys"}


# ----------------------------------------------------------- host-inclusive
def _hip():
    L = C.CDLL("libamdhip64.so")
    L.hipHostRegister.argtypes = [C.c_void_p, C.c_size_t, C.c_uint]
    L.hipHostRegister.restype = C.c_int
    L.hipHostUnregister.argtypes = [C.c_void_p]
    L.hipHostUnregister.restype = C.c_int
    return L


def _decode_pipeline(torch, lsmgpu, src, off, chunks, nb, reps, bounce):
    """Chunked H2D -> decode -> D2H of the parsed SoA, three streams, double
    buffered.  src: host uint8 tensor over the file (registered pages, or plain
    mmap'd pages when bounce=True: each chunk is then first copied by the CPU
    into a pinned staging buffer).  The SoA copy-back of a chunk is sized from
    its decoded item count (item_start[n], read back one chunk behind).
    Returns (best seconds, host item_start, host fields)."""
    import numpy as np
    pad = lsmgpu.LSM_INPUT_PADDING
    dev = torch.device("cuda")
    max_bytes = max(c[3] for c in chunks)
    max_n = max(c[1] - c[0] for c in chunks)
    cap = max_bytes // 3 + 1  # items of a chunk are bounded by its bytes / 3
    dbuf = [torch.empty(max_bytes, dtype=torch.uint8, device=dev) for _ in range(2)]
    doff = [torch.empty(max_n + 1, dtype=torch.int64, device=dev) for _ in range(2)]
    decs = [lsmgpu.Decoder(dev) for _ in range(2)]
    outs = [decs[k].alloc_outputs(cap, max_n, fields=DATA_FIELDS) for k in range(2)]
    total_cap = int(off[nb]) // 3 + 1
    hout = {f: torch.empty(total_cap, dtype=outs[0][f].dtype).pin_memory() for f in DATA_FIELDS}
    hcnt = torch.empty(len(chunks), dtype=torch.int32).pin_memory()  # items per chunk (item_start[n])
    staging = [torch.empty(max_bytes, dtype=torch.uint8).pin_memory() for _ in range(2)] if bounce else None
    s_in, s_dec, s_out = torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.Stream()
    free = [torch.cuda.Event() for _ in range(2)]        # buffer k reusable (its SoA copied out)
    h2d_done = [torch.cuda.Event() for _ in range(2)]    # staging k consumed by its H2D
    counted = [torch.cuda.Event() for _ in range(2)]     # item_start of chunk in buffer k on the host
    best = None
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        item_base, pending = 0, None

        def drain(p):  # the SoA of a decoded chunk, sized by its item count
            nonlocal item_base
            pk, pi = p
            counted[pk].synchronize()
            ni = int(hcnt[pi])
            with torch.cuda.stream(s_out):
                for f in DATA_FIELDS:
                    hout[f][item_base:item_base + ni].copy_(outs[pk][f][:ni], non_blocking=True)
                free[pk].record(s_out)
            item_base += ni

        for i, (b0, b1, s0, nbytes, rel) in enumerate(chunks):
            k = i % 2
            n = b1 - b0
            with torch.cuda.stream(s_in):
                if i >= 2:
                    s_in.wait_event(free[k])
                if bounce:
                    h2d_done[k].synchronize()  # staging k free again
                    staging[k][:nbytes].copy_(src[s0:s0 + nbytes])  # page cache -> pinned (CPU)
                    dbuf[k][:nbytes].copy_(staging[k][:nbytes], non_blocking=True)
                    h2d_done[k].record(s_in)
                else:
                    dbuf[k][:nbytes].copy_(src[s0:s0 + nbytes], non_blocking=True)
                doff[k][:n + 1].copy_(rel, non_blocking=True)
            s_dec.wait_stream(s_in)
            decs[k].decode(dbuf[k], doff[k], n, outs[k], cap, stream=s_dec)
            s_out.wait_stream(s_dec)
            with torch.cuda.stream(s_out):
                hcnt[i:i + 1].copy_(outs[k]["item_start"][n:n + 1], non_blocking=True)
                counted[k].record(s_out)
            if pending is not None:
                drain(pending)
            pending = (k, i)
        drain(pending)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        best = el if best is None else min(best, el)
    return best, hcnt, hout, item_base


def host_inclusive_decode(torch, lsmgpu, enc, nb_all, ipb=52, max_blocks=262144, chunk_blocks=32768, reps=2):
    """Blocks start in an mmap'd SST file (the Scanner / compaction read side):
    chunked H2D -> decode -> D2H of the parsed SoA (sized from each chunk's
    decoded item count) on three streams, double-buffered, two ways:
      registered  the file's mapped pages hipHostRegister'ed (DMA straight from
                  the page cache); the registration is timed and reported both
                  apart and included (a reader registers each file once);
      bounce      no registration: each chunk copied by the CPU from the mapped
                  pages into a pinned staging buffer, then DMA'd.
    The file was just written, so its pages are in the page cache (no disk read)."""
    import numpy as np
    nb = min(max_blocks, nb_all)
    off = enc["block_off"][:nb + 1].cpu().numpy().astype(np.int64)
    total = int(off[-1])
    pad = lsmgpu.LSM_INPUT_PADDING
    fd, path = tempfile.mkstemp(prefix="lsm_sst_", dir="/tmp")
    res = {"blocks": nb, "bytes": total, "chunk_blocks": chunk_blocks,
           "note": "mmap'd SST file (page-cache warm) -> H2D -> decode -> D2H parsed SoA (25 B/item, sized from "
                   "item_start), 3 streams, double-buffered"}
    try:
        os.write(fd, enc["buf"][:total].cpu().numpy().tobytes() + bytes(pad))  # the GPU-encoded table
        os.fsync(fd)
        size = total + pad
        mm = mmap.mmap(fd, size, mmap.MAP_SHARED, mmap.PROT_READ | mmap.PROT_WRITE)
        hbuf_np = np.frombuffer(mm, dtype=np.uint8)
        hbuf = torch.from_numpy(hbuf_np)
        chunks = []
        for b0 in range(0, nb, chunk_blocks):
            b1 = min(nb, b0 + chunk_blocks)
            s0 = int(off[b0]) & ~15
            rel = torch.from_numpy(off[b0:b1 + 1] - s0).pin_memory()
            chunks.append((b0, b1, s0, int(off[b1]) - s0 + pad, rel))
        # bounce buffers first (no registration), then the registered pages
        t_b, _, hout, n_items = _decode_pipeline(torch, lsmgpu, hbuf, off, chunks, nb, reps, bounce=True)
        assert n_items == nb * ipb and bool((hout["val_len"][:n_items] == 64).all())
        res["bounce"] = {"GiB_per_s": round(total / t_b / 2 ** 30, 3), "ms": round(t_b * 1e3, 3)}
        hip = _hip()
        t0 = time.perf_counter()
        rc = hip.hipHostRegister(hbuf.data_ptr(), size, 0)
        reg_ms = (time.perf_counter() - t0) * 1e3
        if rc == 0:
            t_r, hstart, hout, n_items = _decode_pipeline(torch, lsmgpu, hbuf, off, chunks, nb, reps, bounce=False)
            assert n_items == nb * ipb and bool((hout["seqno"][:n_items] == 63).all())
            t0 = time.perf_counter()
            hip.hipHostUnregister(hbuf.data_ptr())
            unreg_ms = (time.perf_counter() - t0) * 1e3
            res["registered"] = {"GiB_per_s": round(total / t_r / 2 ** 30, 3), "ms": round(t_r * 1e3, 3),
                                 "register_ms": round(reg_ms, 2), "unregister_ms": round(unreg_ms, 2),
                                 "GiB_per_s_incl_registration": round(
                                     total / (t_r + (reg_ms + unreg_ms) * 1e-3) / 2 ** 30, 3)}
        else:
            res["registered"] = {"skipped": f"hipHostRegister returned {rc}"}
        del hbuf, hbuf_np
        mm.close()
    finally:
        os.close(fd)
        os.unlink(path)
    reg = res.get("registered", {})
    res["GiB_per_s"] = max(res["bounce"]["GiB_per_s"], reg.get("GiB_per_s_incl_registration", 0.0))
    return res


def host_inclusive_encode(torch, lsmgpu, items_host, starts_np, nb_all, max_blocks=262144, chunk_blocks=32768,
                          reps=2):
    """Items start in a pinned host write buffer (the flush / compaction output
    side): chunked H2D of the item SoA -> encode -> D2H of the on-disk blocks
    into a pinned host output, three streams, double-buffered."""
    import numpy as np
    nb = min(max_blocks, nb_all)
    n_items = int(starts_np[nb])
    ko, vo = items_host.key_off, items_host.val_off
    hk = torch.from_numpy(items_host.keys[:int(ko[n_items])]).pin_memory()
    hv = torch.from_numpy(items_host.vals[:int(vo[n_items])]).pin_memory()
    hko = torch.from_numpy(ko[:n_items + 1].view(np.int64)).pin_memory()
    hvo = torch.from_numpy(vo[:n_items + 1].view(np.int64)).pin_memory()
    hsq = torch.from_numpy(items_host.seqno[:n_items].view(np.int64)).pin_memory()
    hvt = torch.from_numpy(items_host.vtype[:n_items]).pin_memory()
    hst = torch.from_numpy(starts_np[:nb + 1].astype(np.int32)).pin_memory()
    chunks = []
    for b0 in range(0, nb, chunk_blocks):
        b1 = min(nb, b0 + chunk_blocks)
        i0, i1 = int(starts_np[b0]), int(starts_np[b1])
        chunks.append((b0, b1, i0, i1))
    dev = torch.device("cuda")
    mi = max(c[3] - c[2] for c in chunks)
    mk = max(int(ko[c[3]] - ko[c[2]]) for c in chunks)
    mv = max(int(vo[c[3]] - vo[c[2]]) for c in chunks)
    mb = max(c[1] - c[0] for c in chunks)
    pad = lsmgpu.LSM_INPUT_PADDING
    bufs = [{"keys": torch.zeros(mk + pad, dtype=torch.uint8, device=dev),
             "vals": torch.zeros(mv + pad, dtype=torch.uint8, device=dev),
             "key_off": torch.empty(mi + 1, dtype=torch.int64, device=dev),
             "val_off": torch.empty(mi + 1, dtype=torch.int64, device=dev),
             "seqno": torch.empty(mi, dtype=torch.int64, device=dev),
             "vtype": torch.empty(mi, dtype=torch.uint8, device=dev),
             "starts": torch.empty(mb + 1, dtype=torch.int32, device=dev)} for _ in range(2)]
    encs = [lsmgpu.Encoder(dev) for _ in range(2)]
    outs = [None, None]
    hout = torch.empty(int(ko[n_items]) + int(vo[n_items]) + 64 * nb + 4096, dtype=torch.uint8).pin_memory()
    hoff = torch.empty(nb + 1, dtype=torch.int64).pin_memory()
    s_in, s_enc, s_out = torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.Stream()
    free = [torch.cuda.Event() for _ in range(2)]
    # output placement: a chunk's encoded size is only known after its encode; the host stream
    # waits for the chunk's last block offset (8 B) before issuing its D2H (pipelined one chunk behind)
    best = None
    written = 0
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        pos = 0
        pending = None
        for i, (b0, b1, i0, i1) in enumerate(chunks):
            k = i % 2
            n, ni = b1 - b0, i1 - i0
            kb, vb = int(ko[i0]), int(vo[i0])
            with torch.cuda.stream(s_in):
                if i >= 2:
                    s_in.wait_event(free[k])
                d = bufs[k]
                d["keys"][:int(ko[i1]) - kb].copy_(hk[kb:int(ko[i1])], non_blocking=True)
                d["vals"][:int(vo[i1]) - vb].copy_(hv[vb:int(vo[i1])], non_blocking=True)
                d["key_off"][:ni + 1].copy_(hko[i0:i1 + 1], non_blocking=True)
                d["val_off"][:ni + 1].copy_(hvo[i0:i1 + 1], non_blocking=True)
                d["seqno"][:ni].copy_(hsq[i0:i1], non_blocking=True)
                d["vtype"][:ni].copy_(hvt[i0:i1], non_blocking=True)
                d["starts"][:n + 1].copy_(hst[b0:b1 + 1], non_blocking=True)
                d["key_off"][:ni + 1].sub_(kb)
                d["val_off"][:ni + 1].sub_(vb)
                d["starts"][:n + 1].sub_(i0)
            s_enc.wait_stream(s_in)
            it = {"keys": d["keys"], "vals": d["vals"], "key_off": d["key_off"][:ni + 1],
                  "val_off": d["val_off"][:ni + 1], "seqno": d["seqno"][:ni], "vtype": d["vtype"][:ni]}
            outs[k] = encs[k].encode(it, d["starts"][:n + 1], n, out=outs[k], stream=s_enc)
            s_out.wait_stream(s_enc)
            if pending is not None:  # D2H of the previous chunk, now that its size is on the host
                pk, pn, pb0 = pending
                torch.cuda.current_stream().synchronize()
                s_out.synchronize()
                sz = int(hoff[pb0 + pn].item())
                with torch.cuda.stream(s_out):
                    hout[pos:pos + sz].copy_(outs[pk]["buf"][:sz], non_blocking=True)
                    free[pk].record(s_out)
                pos += sz
            with torch.cuda.stream(s_out):
                hoff[b0:b1 + 1].copy_(outs[k]["block_off"][:n + 1], non_blocking=True)
            pending = (k, n, b0)
        s_out.synchronize()
        pk, pn, pb0 = pending
        sz = int(hoff[pb0 + pn].item())
        with torch.cuda.stream(s_out):
            hout[pos:pos + sz].copy_(outs[pk]["buf"][:sz], non_blocking=True)
        torch.cuda.synchronize()
        pos += sz
        el = time.perf_counter() - t0
        best = el if best is None else min(best, el)
        written = pos
    return {"GiB_per_s": round(written / best / 2 ** 30, 3), "ms": round(best * 1e3, 3), "blocks": nb,
            "bytes_out": written, "chunk_blocks": chunk_blocks,
            "note": "pinned host item SoA -> H2D -> encode -> D2H on-disk blocks, 3 streams, double-buffered; "
                    "rate = encoded bytes / wall"}


def load_traffic(kernel, n_blocks):
    """HBM bytes of one launch of `kernel` over n_blocks, from the newest committed
    rocprofv3 PMC summary (profiles/traffic_*.json), scaled per block."""
    best, src = None, None
    for p in sorted((ROOT / "profiles").glob("traffic_*.json")):
        try:
            d = json.loads(p.read_text())
        except Exception:
            continue
        entry = d.get(kernel) if isinstance(d, dict) and kernel in d else (d if d.get("kernel") == kernel else None)
        if entry:
            best, src = entry, p.name
    if not best:
        return None, None
    return int(round(best["bytes_per_launch"] * n_blocks / best["blocks"])), f"{src} ({best['blocks']} blocks)"


def roofline_entry(name, alg_bytes, ms, ceil, traffic_kernel, nb):
    achieved = alg_bytes / (ms * 1e-3) / 1e9
    traffic, src = load_traffic(traffic_kernel, nb)
    return {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": traffic, "traffic_source": src,
            "kernel": name, "kernel_ms": round(ms, 4), "alg_bytes_per_launch": alg_bytes,
            "practical_peak": ceil, "frac_of_copy_ceiling": round(achieved / ceil["copy_GBps"], 4) if ceil else None}


_LIB_SHA = None


def lib_sha256():
    """sha256 of the product library this process loaded (lsmgpu.LIB_PATH)."""
    global _LIB_SHA
    if _LIB_SHA is None:
        import hashlib
        import lsmgpu
        _LIB_SHA = hashlib.sha256(Path(lsmgpu.LIB_PATH).read_bytes()).hexdigest()
    return _LIB_SHA


def load_trace_ms(kernels, n_blocks):
    """Mean duration (ms) of one launch of each (kernel, workgroups) pair, summed,
    from a committed rocprofv3 kernel-trace summary
    (profiles/*_bench_kernels_by_grid.csv, scripts/trace_by_grid.py) of a bench
    run over the same batch size BY THE SAME LIBRARY BUILD: the trace's sidecar
    (*.lib.json, written by scripts/profile_round.sh) must carry the sha256 of
    the liblsmgpu.so this process loaded.  None otherwise (a trace of an older
    build would report stale kernel times beside the live ones)."""
    import csv
    best, src = None, None
    for p in sorted((ROOT / "profiles").glob("*_bench_kernels_by_grid.csv")):  # (round names sort in order)
        side = p.with_name(p.name.replace(".csv", ".lib.json"))
        try:
            if json.loads(side.read_text()).get("lib_sha256") != lib_sha256():
                continue
            rows = list(csv.DictReader(p.open()))
        except Exception:
            continue
        if not rows or not {"kernel", "workgroups"} <= set(rows[0]) or not ({"avg_us", "avg_ns"} & set(rows[0])):
            continue
        by = {(r["kernel"], int(r["workgroups"])): r for r in rows}
        if not all(k in by for k in kernels):
            continue
        unit = 1e-3 if "avg_us" in rows[0] else 1e-6
        col = "avg_us" if "avg_us" in rows[0] else "avg_ns"
        best, src = sum(float(by[k][col]) * unit for k in kernels), p.name
    return (round(best, 4), src) if best is not None else (None, None)


def encode_roofline(name, enc_ms, key_val, n_items, nb, total_bytes, ceil, trace_kernels=None, off_bytes=8):
    """Encode roofline.  `achieved` / `frac` count SURVEY §8(d)'s algorithmic
    bytes (the key and value bytes, 17 B of item SoA per item with 4-byte
    offsets, the blocks written); `achieved_abi` / `frac_abi` count what the
    call's ABI reads and writes (off_bytes-wide key / value offsets: 25 B of SoA
    per item with lsm_items' u64 offsets, 17 B with lsm_items32's u32 ones, plus
    block_item_start, block_off and status).  kernel_ms is the whole encode call
    timed with HIP events on its launch stream (plan + scan + write kernels);
    kernel_ms_trace the same kernels' mean launch durations from a committed
    rocprofv3 trace of this very library build, when one exists."""
    enc_alg_abi = key_val + n_items * (ENC_IN_PER_ITEM - 2 * (8 - off_bytes)) + 4 * (nb + 1) + total_bytes + \
        8 * (nb + 1) + 4 * nb
    enc_alg_survey = key_val + n_items * ENC_IN_PER_ITEM_SURVEY + total_bytes
    r = roofline_entry(name, enc_alg_survey, enc_ms, ceil, "lsm_encode_blocks", nb)
    r["alg_bytes_source"] = "SURVEY 8(d): key + value bytes + 17 B/item SoA (4-B offsets) + blocks written"
    r["kernel_ms_source"] = "HIP events around the whole encode call on its launch stream"
    r["alg_bytes_abi"] = enc_alg_abi
    r["achieved_abi"] = round(enc_alg_abi / (enc_ms * 1e-3) / 1e9, 1)
    r["frac_abi"] = round(enc_alg_abi / (enc_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4)
    if trace_kernels:
        tms, tsrc = load_trace_ms(trace_kernels, nb)
        if tms:
            r["kernel_ms_trace"] = tms
            r["kernel_ms_trace_source"] = tsrc
            r["frac_trace"] = round(enc_alg_survey / (tms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4)
            r["frac_abi_trace"] = round(enc_alg_abi / (tms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4)
    return r


def bench_random_keys(torch, lsmgpu, steps, rank, threads, ceil, nb=1 << 20):
    """SURVEY §8(d) config 2 variant G2: the headline shape with random 16 B
    keys (sorted), 64 B values, 1 M x 4 KiB blocks (~4466 B each: 0-4 key
    bytes shared with the restart head).  Encode and decode timed alone, each
    with its roofline; every block checked against the oracle."""
    check_cut_rule(lsmgpu, 52, 16, 64)
    items, starts, n = make_workload(torch, lsmgpu, nb, seed=0x5EED0012 + rank, kind="random")
    enc_ctx = lsmgpu.Encoder()
    enc = enc_ctx.encode(items, starts, nb)
    torch.cuda.synchronize()
    total = int(enc["block_off"][nb].item())
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    enc_ctx.encode(items, starts, nb, out=enc)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(steps):
        enc_ctx.encode(items, starts, nb, out=enc)
    e1.record()
    torch.cuda.synchronize()
    enc_ms = e0.elapsed_time(e1) / steps
    dec_ms, out = time_decode(torch, lsmgpu, enc["buf"], enc["block_off"], nb, n, steps)
    dec = lsmgpu.Decoder(enc["buf"].device)
    out2 = dec.alloc_outputs(n, nb)
    kdec = lambda: dec.decode(enc["buf"], enc["block_off"], nb, out2, n,  # noqa: E731
                              tuning=(0, 0, 0, lsmgpu.DECODE_ITEM_START_VALID))
    out2["item_start"].copy_(out["item_start"])
    kdec()
    torch.cuda.synchronize()
    e0.record()
    for _ in range(steps):
        kdec()
    e1.record()
    torch.cuda.synchronize()
    kdec_ms = e0.elapsed_time(e1) / steps
    ref_buf, ref_off = check_encode_all(torch, items, starts, enc, nb, n, threads)
    check_decode_all(out, ref_buf, ref_off, nb, threads)
    check_decode_all(out2, ref_buf, ref_off, nb, threads)
    key_val = int(items["key_off"][n].item()) + int(items["val_off"][n].item())
    dec_alg = total + n * PARSED_BYTES_PER_ITEM + nb * PER_BLOCK_OUT
    r_dec = roofline_entry("decode_blocks_kernel (item_start precomputed)", dec_alg, kdec_ms, ceil,
                           "decode_blocks_kernel", nb)
    r_dec["traffic"] = r_dec["traffic_source"] = None  # (the committed PMC summaries are of the G1 batch)
    r_dec["read_only_frac"] = round(total / (kdec_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4)
    r_enc = encode_roofline("lsm_encode_blocks (encode_plan_wave_kernel + scan + encode_group_kernel)", enc_ms,
                            key_val, n, nb, total, ceil)
    r_enc["traffic"] = r_enc["traffic_source"] = None
    res = {"workload": "SURVEY §8(d) config 2 variant G2: 1 M x 4 KiB blocks, random sorted 16 B keys, 64 B values, "
                       "seqno 63, restart interval 16",
           "blocks": nb, "items": n, "bytes": total,
           "encode_ms": round(enc_ms, 4), "encode_GiB_per_s": round(total / (enc_ms * 1e-3) / 2 ** 30, 3),
           "decode_ms": round(dec_ms, 4), "decode_kernel_ms": round(kdec_ms, 4),
           "decode_GiB_per_s": round(total / (dec_ms * 1e-3) / 2 ** 30, 3),
           "round_trip_GiB_per_s": round(total / ((enc_ms + dec_ms) * 1e-3) / 2 ** 30, 3),
           "roofline_decode": r_dec, "roofline_encode": r_enc, "oracle_checked_blocks": nb}
    del items, enc, out, out2, ref_buf
    torch.cuda.empty_cache()
    return res


# --------------------------------------------------------------------- main
def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--blocks", type=int, default=1 << 20)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-host", action="store_true", help="skip the host-inclusive (PCIe) measurements")
    ap.add_argument("--cpu-seconds", type=float, default=2.0, help="minimum seconds per CPU baseline leg")
    ap.add_argument("--skip-verify", action="store_true", help="(profiling only) skip the full oracle checks")
    ap.add_argument("--no-extra", action="store_true", help="skip the configs[3]/[4] and side legs")
    args = ap.parse_args()

    import numpy as np
    import torch
    import lsmgpu

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    # LSM_BENCH_REHEARSE=1: rehearse the N > 1 path on a one-GPU box (every
    # rank on cuda:0, the two timing reductions over gloo on the host); never
    # set by the driver, whose N > 1 runs use one GPU per rank and RCCL
    rehearse = world > 1 and os.environ.get("LSM_BENCH_REHEARSE") == "1"
    # LSM_BENCH_DIST=1 under torchrun --nproc-per-node 1: a one-rank RCCL group,
    # so the N > 1 code path (RCCL init, device barriers, the two device
    # all_reduces) runs on a one-GPU box; the result equals the N = 1 run
    if world > 1 or os.environ.get("LSM_BENCH_DIST") == "1":
        import torch.distributed as dist
        if rehearse:
            torch.cuda.set_device(0)
            dist.init_process_group("gloo")
        else:
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())
    red_dev = torch.device("cpu") if rehearse else dev  # where the timing / byte reductions run
    threads = max(1, HOST_THREADS // world) if rehearse else host_threads(world)  # (rehearsal: one GPU's CPU share)

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    nb = args.blocks
    check_cut_rule(lsmgpu, 52, 16, 64)
    t_gen = time.perf_counter()
    items, starts, n_items = make_workload(torch, lsmgpu, nb, seed=0x5EED0002 + rank)
    # the timed step encodes through lsm_encode_blocks32 (u32 key / value offsets: SURVEY 8(d)'s
    # 4 + 4 B per item; the arenas are < 4 GiB); the u64-offset lsm_encode_blocks is timed beside it
    items32 = dict(items, key_off=items["key_off"].to(torch.int32), val_off=items["val_off"].to(torch.int32))
    encoder = lsmgpu.Encoder(dev)
    enc = encoder.encode(items, starts, nb)
    torch.cuda.synchronize()
    total_bytes = int(enc["block_off"][nb].item())
    dec_ctx = lsmgpu.Decoder(dev)
    out = dec_ctx.alloc_outputs(n_items, nb, fields=DATA_FIELDS)
    log(f"[rank {rank}] generated+encoded {nb} blocks, {n_items} items, {total_bytes / 2**30:.3f} GiB "
        f"in {time.perf_counter() - t_gen:.1f}s")

    def step():
        encoder.encode(items32, starts, nb, out=enc)
        dec_ctx.decode(enc["buf"], enc["block_off"], nb, out, n_items)

    step()
    torch.cuda.synchronize()
    ref_buf = ref_off = items_host = starts_np = None
    if not args.skip_verify:
        t_chk = time.perf_counter()
        ref_buf, ref_off = check_encode_all(torch, items, starts, enc, nb, n_items, threads)
        check_decode_all(out, ref_buf, ref_off, nb, threads)
        items_host = host_items(items, n_items)
        starts_np = starts.cpu().numpy().astype(np.uint32)
        log(f"[rank {rank}] all {nb} blocks bit-exact vs the oracle (encode bytes + decoded fields) "
            f"in {time.perf_counter() - t_chk:.1f}s")

    for _ in range(args.warmup):
        step()
    barrier()
    t0 = time.perf_counter()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(args.steps):
        step()
    e1.record()
    barrier()
    el = time.perf_counter() - t0
    gpu_ms = e0.elapsed_time(e1)
    if dist is not None:
        t = torch.tensor([el], dtype=torch.float64, device=red_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
        tb = torch.tensor([total_bytes], dtype=torch.int64, device=red_dev)
        dist.all_reduce(tb, op=dist.ReduceOp.SUM)
        all_bytes = int(tb.item())
    else:
        all_bytes = total_bytes
    ms_per_step = el * 1e3 / args.steps
    value = all_bytes * args.steps / el / 2 ** 30

    # each direction alone, HIP events on its launch stream
    def timed(fn, reps):
        fn()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            fn()
        b.record()
        torch.cuda.synchronize()
        return a.elapsed_time(b) / reps

    reps = max(5, args.steps // 2)
    enc_ms = timed(lambda: encoder.encode(items32, starts, nb, out=enc), reps)
    enc64_ms = timed(lambda: encoder.encode(items, starts, nb, out=enc), reps)  # (u64 offsets: the same bytes)
    dec_ms = timed(lambda: dec_ctx.decode(enc["buf"], enc["block_off"], nb, out, n_items), reps)
    kdec_ms = timed(lambda: dec_ctx.decode(enc["buf"], enc["block_off"], nb, out, n_items,
                                           tuning=(0, 0, 0, lsmgpu.DECODE_ITEM_START_VALID)), reps)
    # the compact 19 B/item layout (lsm_decode_blocks16), same blocks, checked against the 32-bit output
    out16 = dec_ctx.alloc_outputs(n_items, nb, compact=True)
    dec_ctx.decode(enc["buf"], enc["block_off"], nb, out16, n_items, compact=True)
    torch.cuda.synchronize()
    assert int((out16["status"][:nb] != 0).sum()) == 0, "compact decode: a block failed"
    for f in ("key_off", "val_off", "val_len"):
        assert torch.equal(out[f][:n_items].to(torch.int64), out16[f][:n_items].to(torch.int64) & 0xFFFF), f
    for f in ("seqno", "key_len", "prefix_len", "vtype"):
        assert torch.equal(out[f][:n_items], out16[f][:n_items]), f
    kdec16_ms = timed(lambda: dec_ctx.decode(enc["buf"], enc["block_off"], nb, out16, n_items, compact=True,
                                             tuning=(0, 0, 0, lsmgpu.DECODE_ITEM_START_VALID)), reps)
    del out16
    ceil = ceilings(torch) if rank == 0 else None
    dec_alg = total_bytes + n_items * PARSED_BYTES_PER_ITEM + nb * PER_BLOCK_OUT
    dec16_alg = total_bytes + n_items * 19 + nb * PER_BLOCK_OUT
    key_val = int(items["key_off"][n_items].item()) + int(items["val_off"][n_items].item())
    r_dec = roofline_entry("decode_blocks_kernel (item_start precomputed)", dec_alg, kdec_ms, ceil,
                           "decode_blocks_kernel", nb)
    r_dec["kernel_ms_source"] = "HIP events around lsm_decode_blocks with item_start precomputed (the decode kernel alone)"
    r_dec["read_only_frac"] = round(total_bytes / (kdec_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4)
    tms, tsrc = load_trace_ms([("decode_blocks_kernel<true, false>", (nb + 53) // 54)], nb) if nb == 1 << 20 \
        else (None, None)
    if tms:
        r_dec["kernel_ms_trace"], r_dec["kernel_ms_trace_source"] = tms, tsrc
        r_dec["read_only_frac_trace"] = round(total_bytes / (tms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4)
    r_enc = encode_roofline("lsm_encode_blocks32 (encode_plan_wave_kernel + scan + encode_group_kernel)", enc_ms,
                            key_val, n_items, nb, total_bytes, ceil, off_bytes=4, trace_kernels=
                            [("encode_plan_wave_kernel<false, 4>", (nb + 127) // 128),
                             ("encode_group_kernel<false, false, false, 4, false>", (nb + 31) // 32)] if nb == 1 << 20 else None)
    dominant = r_enc if enc_ms >= kdec_ms else r_dec

    extra = {}
    if not args.no_extra:
        extra["point_read"] = bench_point_read(torch, lsmgpu, items, enc, nb, n_items)
        extra["file_checksum"] = bench_file_checksum(torch, lsmgpu, enc, total_bytes)
        if rank == 0:
            extra["file_checksum_batch"] = bench_file_checksum_batch(torch, lsmgpu, enc, total_bytes)
        extra["bloom"] = bench_bloom(torch, lsmgpu, items, n_items)
        if rank == 0:
            extra["lz4"] = bench_lz4(torch, lsmgpu, enc, nb)
        mkeys, extra["materialize"] = bench_materialize(torch, lsmgpu, enc, nb, out, n_items)
        assert torch.equal(mkeys, items["keys"][:n_items * 16]), "materialize: keys differ from the encoder input"
        del mkeys
        if rank == 0 and world == 1:
            extra["table_scan"] = bench_table_scan(torch, lsmgpu, items, enc, nb, n_items, out)
            torch.cuda.empty_cache()
    hostinc = {}
    if rank == 0 and world == 1 and not args.no_host and ref_buf is not None:
        hostinc["decode_from_mmap"] = host_inclusive_decode(torch, lsmgpu, enc, nb)
        hostinc["encode_from_host_buffer"] = host_inclusive_encode(torch, lsmgpu, items_host, starts_np, nb)
    del out, items
    torch.cuda.empty_cache()
    if not args.no_extra and not args.skip_verify:
        if world == 1:
            extra["config4"] = bench_config4(torch, lsmgpu, max(3, args.steps // 4), rank, threads)
        extra["config5"] = bench_config5(torch, lsmgpu, max(3, args.steps // 4), rank, world, dist, red_dev, threads)
        if world == 1:
            extra["large_blocks"] = bench_large_blocks(torch, lsmgpu, threads)
            extra["hash_index"] = bench_hash_index(torch, lsmgpu, max(3, args.steps // 4), threads)
            extra["random_keys"] = bench_random_keys(torch, lsmgpu, max(3, args.steps // 4), rank, threads, ceil)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu and ref_buf is not None:
        cpu = cpu_baseline(ref_buf, ref_off, items_host, starts_np, min_seconds=args.cpu_seconds)

    if rank == 0:
        verified = "skipped" if args.skip_verify else f"all {nb} blocks per rank bit-exact vs the oracle (encoded bytes " \
                                                      f"and every decoded field)"
        line = {
            "metric": BASELINE_METRIC,
            "value": round(value, 3),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": f"synthetic (16 B BE-counter keys, 64 B random values, seqno 63); {verified}",
            "config": {"workload": "BASELINE configs[1]/[2]: encode + decode round trip of 1 M x 4 KiB data blocks, "
                                   "device-resident",
                       "blocks_per_gpu": nb, "items_per_gpu": n_items, "block_bytes_per_gpu": total_bytes,
                       "restart_interval": 16, "hash_ratio": 0.0, "key_len": 16, "val_len": 64,
                       "step": "lsm_encode_blocks32 (item SoA, u32 offsets -> blocks) + lsm_decode_blocks "
                               "(blocks -> parsed SoA)",
                       "parallelism": f"shard{world} (independent block batches, no collective)"},
            "roofline": dominant,
            "roofline_decode": r_dec,
            "roofline_encode": r_enc,
            "cpu_baseline": cpu,
            "encode": {"ms": round(enc_ms, 4), "GiB_per_s_written": round(total_bytes / (enc_ms * 1e-3) / 2 ** 30, 3),
                       "entry": "lsm_encode_blocks32 (u32 key / value offsets)",
                       "u64_offsets_ms": round(enc64_ms, 4),
                       "u64_offsets_note": "lsm_encode_blocks (lsm_items, u64 offsets) on the same items: same bytes"},
            "decode": {"ms": round(dec_ms, 4), "GiB_per_s": round(total_bytes / (dec_ms * 1e-3) / 2 ** 30, 3),
                       "kernel_ms": round(kdec_ms, 4),
                       "note": "whole lsm_decode_blocks call (trailer counts + scan + decode kernel)"},
            "decode_compact": {"kernel_ms": round(kdec16_ms, 4), "alg_bytes": dec16_alg,
                               "GBps_alg": round(dec16_alg / (kdec16_ms * 1e-3) / 1e9, 1),
                               "read_only_frac": round(total_bytes / (kdec16_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
                               "note": "lsm_decode_blocks16 (19 B/item: u16 payload offsets / lengths), item_start "
                                       "precomputed; every field equal to the 32-bit decode's"},
            "round_trip_traffic_GiB_per_s": round(2 * value, 3),
            **extra,
            "host_inclusive": hostinc or None,
            "gpu_event_ms_per_step": round(gpu_ms / args.steps, 4),
        }
        if rehearse:  # every rank on cuda:0: a rehearsal of the N > 1 path, never a multi-GPU measurement
            line["rehearsal"] = True
            line["physical_gpus"] = 1
            line["data"] += f"; REHEARSAL: {world} ranks shared one GPU, not a multi-GPU measurement"
        if dist is not None:
            line["process_group"] = {"backend": dist.get_backend(), "world_size": dist.get_world_size()}
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
