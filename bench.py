#!/usr/bin/env python3
"""bench.py — BASELINE.json headline: device-resident data-block decode GiB/s,
1 M x 4 KiB blocks, 16 B keys / 64 B values (configs[1]).

A "step" = one lsm_decode_blocks call over the whole batch of on-disk blocks
already resident in HBM: trailer item counts + scan + verify (header and
xxh3_128) + parse of every record into the parsed-item SoA.  value = total
block bytes decoded by all ranks / (max over ranks of the timed K steps).

Synthetic input: keys = 16 B big-endian counters, values 64 B
uniform random, seqno 63, all Value, cut by the writer rule at 4096 B
(52 items / 3769-3773 B per block), restart interval 16, hash ratio 0.
The blocks are produced by the GPU encoder (lsm_encode_blocks) and a sample is
checked bit-exactly against the oracle before timing.

N > 1: one process per GPU (torch.distributed, RCCL), each rank decodes its own
1 M-block shard (weak scaling, no data-path collective).

Side legs in the same JSON line (not `value`): encode and the configs[2] round
trip, configs[3] (prefix-heavy 16 KiB blocks, N = 1), configs[4] (8 GiB of
mixed 4/16/64 KiB data + index blocks byte-split across the ranks: strong
scaling), batched point reads, the whole-file checksum, the host-inclusive
(PCIe) decode rate and the CPU baseline (oracle port on the host cores).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
for p in (ROOT / "lsm-tree_amd", ROOT / "oracle", ROOT / "tests"):
    sys.path.insert(0, str(p))

BASELINE_METRIC = "device-resident data-block decode+encode GiB/s, 1 M \u00d7 4 KiB blocks"  # BASELINE.json
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec, /opt/skills/guides/MI355X_MICROARCH.md
PARSED_BYTES_PER_ITEM = 8 + 4 + 4 + 4 + 2 + 2 + 1  # seqno key_off val_off val_len key_len prefix_len vtype
PER_BLOCK_OUT = 8  # item_start u32 + status i32


def log(*a):
    print(*a, file=sys.stderr, flush=True)


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


def verify_sample(torch, lsmgpu, items, starts, enc, dec, n_blocks, n_items, rank):
    """Bit-exact check of sampled blocks against the oracle + size-independent
    properties of the full batch (all statuses OK, item count, round trip)."""
    import numpy as np
    import pyoracle

    st_enc = enc["status"][:n_blocks]
    st_dec = dec["status"][:n_blocks]
    assert int((st_enc != 0).sum().item()) == 0, "encode status"
    assert int((st_dec != 0).sum().item()) == 0, "decode status"
    assert int(dec["item_start"][n_blocks].item()) == n_items, "item count"
    # decoded seqnos / lengths equal the encoded input everywhere
    assert bool((dec["seqno"][:n_items] == items["seqno"]).all().item())
    assert bool((dec["val_len"][:n_items] == 64).all().item())
    # a sample of blocks: GPU bytes == oracle bytes, GPU parsed fields == oracle
    rng = np.random.default_rng(rank + 1)
    picks = sorted(set(rng.integers(0, n_blocks, 64).tolist()) | {0, n_blocks - 1})
    off = enc["block_off"]
    for b in picks:
        s0, s1 = int(starts[b].item()), int(starts[b + 1].item())
        ko = items["key_off"][s0:s1 + 1].cpu().numpy().astype(np.uint64)
        vo = items["val_off"][s0:s1 + 1].cpu().numpy().astype(np.uint64)
        kb = items["keys"][int(ko[0]):int(ko[-1])].cpu().numpy()
        vb = items["vals"][int(vo[0]):int(vo[-1])].cpu().numpy()
        it = pyoracle.Items(kb, ko - ko[0], vb, vo - vo[0], items["seqno"][s0:s1].cpu().numpy().view(np.uint64),
                            items["vtype"][s0:s1].cpu().numpy())
        ref = pyoracle.block_write(pyoracle.data_block_encode(it, 0, s1 - s0))
        o0, o1 = int(off[b].item()), int(off[b + 1].item())
        got = enc["buf"][o0:o1].cpu().numpy().tobytes()
        assert got == ref, f"block {b} bytes differ from oracle"
        n, parsed = pyoracle.data_block_decode(ref[33:])
        i0 = int(dec["item_start"][b].item())
        for f, dt in (("seqno", np.uint64), ("key_off", np.uint32), ("val_off", np.uint32),
                      ("key_len", np.uint16), ("prefix_len", np.uint16), ("vtype", np.uint8)):
            gv = dec[f][i0:i0 + n].cpu().numpy().view(dt)
            assert (gv == parsed[f].astype(dt)).all(), (b, f)
    return len(picks)


def cpu_baseline(torch, enc, n_blocks, min_seconds=10.0, sample_blocks=65536, threads=None):
    """Oracle (scalar C port of the reference path) on the host cores: verify +
    full forward parse of a bounded sample, repeated for >= min_seconds."""
    import numpy as np
    import pyoracle

    nb = min(sample_blocks, n_blocks)
    off = enc["block_off"][:nb + 1].cpu().numpy().view(np.uint64).copy()
    blocks = enc["buf"][:int(off[-1])].cpu().numpy()
    threads = threads or min(16, os.cpu_count() or 1)
    nbytes = int(off[-1])
    passes, t0 = 0, time.perf_counter()
    while True:
        parsed, item_start, status = pyoracle.decode_blocks(blocks, off, nthreads=threads)
        passes += 1
        el = time.perf_counter() - t0
        if el >= min_seconds or passes >= 2000:
            break
    assert (status == 0).all()
    return {"value": round(nbytes * passes / el / 2 ** 30, 3), "unit": "GiB/s", "cores": threads, "kind": "port",
            "sample": f"{nb} blocks ({nbytes / 1e6:.1f} MB) of the same batch, {passes} passes in {el:.1f} s: "
                      f"header+xxh3_128 verify and full forward parse (oracle/batch.c)"}


DATA_FIELDS = ["seqno", "key_off", "val_off", "val_len", "key_len", "prefix_len", "vtype"]


def host_inclusive(torch, lsmgpu, enc, item_start, nb, chunk_blocks=131072, reps=2):
    """Blocks start in pinned host memory (the mmap'd-SST case): chunked,
    double-buffered H2D copy -> decode -> D2H of the parsed SoA on three
    streams.  Returns input GiB/s over the whole pipeline (not `value`)."""
    import numpy as np
    off = enc["block_off"][:nb + 1].cpu().numpy().astype(np.int64)
    ist = item_start[:nb + 1].cpu().numpy().astype(np.int64)
    total = int(off[-1])
    pad = lsmgpu.LSM_INPUT_PADDING
    hbuf = torch.empty(total + pad, dtype=torch.uint8).pin_memory()
    hbuf.copy_(enc["buf"][:total + pad].cpu())
    chunks = []
    for b0 in range(0, nb, chunk_blocks):
        b1 = min(nb, b0 + chunk_blocks)
        s0 = int(off[b0]) & ~15
        rel = torch.from_numpy(off[b0:b1 + 1] - s0).pin_memory()
        chunks.append((b0, b1, s0, int(off[b1]) - s0 + pad, rel, int(ist[b0]), int(ist[b1] - ist[b0])))
    max_bytes = max(c[3] for c in chunks)
    max_n = max(c[1] - c[0] for c in chunks)
    cap = max(c[6] for c in chunks)
    dev = enc["buf"].device
    dbuf = [torch.empty(max_bytes, dtype=torch.uint8, device=dev) for _ in range(2)]
    doff = [torch.empty(max_n + 1, dtype=torch.int64, device=dev) for _ in range(2)]
    decs = [lsmgpu.Decoder(dev) for _ in range(2)]
    outs = [decs[k].alloc_outputs(cap, max_n, fields=DATA_FIELDS) for k in range(2)]
    hout = {f: torch.empty(int(ist[-1]) + 1, dtype=outs[0][f].dtype).pin_memory() for f in DATA_FIELDS}
    s_in, s_dec, s_out = torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.Stream()
    free = [torch.cuda.Event() for _ in range(2)]
    best = None
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i, (b0, b1, s0, nbytes, rel, i0, ni) in enumerate(chunks):
            k = i % 2
            n = b1 - b0
            with torch.cuda.stream(s_in):
                if i >= 2:
                    s_in.wait_event(free[k])
                dbuf[k][:nbytes].copy_(hbuf[s0:s0 + nbytes], non_blocking=True)
                doff[k][:n + 1].copy_(rel, non_blocking=True)
            s_dec.wait_stream(s_in)
            decs[k].decode(dbuf[k], doff[k], n, outs[k], cap, stream=s_dec)
            s_out.wait_stream(s_dec)
            with torch.cuda.stream(s_out):
                for f in DATA_FIELDS:
                    hout[f][i0:i0 + ni].copy_(outs[k][f][:ni], non_blocking=True)
                free[k].record(s_out)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        best = el if best is None else min(best, el)
    # the host copy of the parsed SoA equals the device-resident decode
    assert bool((hout["val_len"][:int(ist[-1])] == 64).all()) and bool((hout["seqno"][:int(ist[-1])] == 63).all())
    return {"GiB_per_s": round(total / best / 2 ** 30, 3), "ms": round(best * 1e3, 3), "chunk_blocks": chunk_blocks,
            "note": "pinned host blocks -> H2D -> decode -> D2H parsed SoA (25 B/item), 3 streams, double-buffered"}


def check_blocks_vs_oracle(torch, items, starts, enc, picks, restart_interval=16):
    """Encoded bytes of the picked blocks == oracle encode of the same items."""
    import numpy as np
    import pyoracle
    off = enc["block_off"]
    for b in picks:
        s0, s1 = int(starts[b].item()), int(starts[b + 1].item())
        ko = items["key_off"][s0:s1 + 1].cpu().numpy().astype(np.uint64)
        vo = items["val_off"][s0:s1 + 1].cpu().numpy().astype(np.uint64)
        it = pyoracle.Items(items["keys"][int(ko[0]):int(ko[-1])].cpu().numpy(), ko - ko[0],
                            items["vals"][int(vo[0]):int(vo[-1])].cpu().numpy(), vo - vo[0],
                            items["seqno"][s0:s1].cpu().numpy().view(np.uint64), items["vtype"][s0:s1].cpu().numpy())
        ref = pyoracle.block_write(pyoracle.data_block_encode(it, 0, s1 - s0, restart_interval=restart_interval))
        got = enc["buf"][int(off[b].item()):int(off[b + 1].item())].cpu().numpy().tobytes()
        assert got == ref, f"block {b} bytes differ from oracle"
    return len(picks)


def time_decode(torch, lsmgpu, blocks, boff, nb, n_items, steps):
    """Device-resident lsm_decode_blocks over a batch (count + scan + verify +
    parse), HIP events on the launch stream; checks every status and the count."""
    dec = lsmgpu.Decoder(blocks.device)
    out = dec.alloc_outputs(n_items, nb, fields=DATA_FIELDS + ["handle_off"])
    dec.decode(blocks, boff, nb, out, n_items)
    torch.cuda.synchronize()
    assert int((out["status"][:nb] != 0).sum().item()) == 0, "decode status"
    assert int(out["item_start"][nb].item()) == n_items, "item count"
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(steps):
        dec.decode(blocks, boff, nb, out, n_items)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / steps, out


def bench_config4(torch, lsmgpu, steps, rank):
    """configs[3]: prefix-heavy keys (32 B shared prefix + 8 B suffix), 256 B
    values, 16 KiB blocks (56 items, 14953 B on disk), 262144 blocks."""
    nb = 262144
    check_cut_rule(lsmgpu, 56, 40, 256, 16384)
    items, starts, n = make_workload(torch, lsmgpu, nb, items_per_block=56, key_len=40, val_len=256,
                                     seed=0x5EED0004 + rank, kind="prefix")
    enc_ctx = lsmgpu.Encoder()
    enc = enc_ctx.encode(items, starts, nb)
    torch.cuda.synchronize()
    assert int((enc["status"][:nb] != 0).sum().item()) == 0
    total = int(enc["block_off"][nb].item())
    assert int(enc["block_off"][1].item()) == 14953  # SURVEY 8 table (first block; later ones vary by a byte)
    checked = check_blocks_vs_oracle(torch, items, starts, enc, [0, 1, nb // 2, nb - 1])
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(3):
        enc_ctx.encode(items, starts, nb, out=enc)
    e1.record()
    torch.cuda.synchronize()
    enc_ms = e0.elapsed_time(e1) / 3
    dec_ms, out = time_decode(torch, lsmgpu, enc["buf"], enc["block_off"], nb, n, steps)
    assert bool((out["prefix_len"][:n].view(torch.int16)[1::56] >= 32).all().item())  # shared 32 B prefix
    res = {"workload": "BASELINE configs[3]: 16 KiB blocks, 32 B shared prefix + 8 B suffix keys, 256 B values",
           "blocks": nb, "bytes": total, "decode_ms": round(dec_ms, 4),
           "decode_GiB_per_s": round(total / (dec_ms * 1e-3) / 2 ** 30, 3),
           "encode_ms": round(enc_ms, 4), "encode_GiB_per_s": round(total / (enc_ms * 1e-3) / 2 ** 30, 3),
           "oracle_checked_blocks": checked}
    del items, enc, out
    torch.cuda.empty_cache()
    return res


# configs[4] mix: equal bytes of 4/16/64 KiB data blocks with counter (G1)
# and random sorted (G2) 16 B keys / 64 B values, plus one full index block
# (RI 1) per 64 MiB "table" (flush target, src/tree/mod.rs:374-377).
C5_SEGMENTS = [(4096, 52, "counter", 3769), (4096, 52, "random", 4466), (16384, 205, "counter", 14636),
               (16384, 205, "random", 17300), (65536, 820, "counter", 58309), (65536, 820, "random", 69219)]
C5_TABLE = 64 << 20


def build_config5_shard(torch, lsmgpu, shard_bytes, rank):
    """This rank's byte share of the configs[4] batch, GPU-encoded: data blocks
    of the six segments, each followed by its index blocks (one per table)."""
    segs, n_items, n_data_blocks, n_index_blocks = [], 0, 0, 0
    picks_checked = 0
    for si, (bs, ipb, kind, est) in enumerate(C5_SEGMENTS):
        nb = max(1, int(shard_bytes / len(C5_SEGMENTS) / est))
        check_cut_rule(lsmgpu, ipb, 16, 64, bs)
        items, starts, n = make_workload(torch, lsmgpu, nb, items_per_block=ipb, seed=0x5EED0005 + 97 * rank + si,
                                         kind=kind)
        enc = lsmgpu.Encoder().encode(items, starts, nb)
        torch.cuda.synchronize()
        assert int((enc["status"][:nb] != 0).sum().item()) == 0
        picks_checked += check_blocks_vs_oracle(torch, items, starts, enc, [0, nb - 1])
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
        assert int((ienc["status"][:nt] != 0).sum().item()) == 0
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
    return blocks, block_off, n_data_blocks + n_index_blocks, n_items, base, n_index_blocks, picks_checked


def bench_config5(torch, lsmgpu, steps, rank, world, dist, dev, total_bytes=8 << 30):
    """configs[4]: 8 GiB of mixed data + index blocks, byte-split across the
    ranks (strong scaling: the batch is fixed, each rank decodes its share)."""
    blocks, boff, nb, n_items, nbytes, n_idx, checked = build_config5_shard(torch, lsmgpu, total_bytes / world, rank)
    ms, out = time_decode(torch, lsmgpu, blocks, boff, nb, n_items, steps)
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
            "oracle_checked_blocks": checked}


def bench_point_read(torch, lsmgpu, items, starts, enc, nb, n_items, n_queries=1 << 20, reps=5):
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
    return {"queries": n_queries, "ms": round(ms, 4), "Mqueries_per_s": round(n_queries / ms / 1e3, 1),
            "note": "lane per query straight from HBM (hash index off: restart binary search + MVCC scan)"}


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


def bench_bloom(torch, lsmgpu, items, n_items, reps=5):
    """Standard Bloom filter over the configs[1] batch's keys (FullFilterWriter,
    src/table/writer/filter/full.rs:47-92, BitsPerKey(10) default): hash64 of every
    key, filter build (k scattered atomicOr per key), then one probe per key.
    Two sizes: one table's worth of keys (1 M, filter 1.25 MB, L2-resident) and
    the whole batch as one filter (HBM-resident)."""
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
    over LZ4 copies of the first `sample` configs[1] blocks: the payloads are
    compressed on the host by liblz4 (pyarrow "lz4_raw", the block format
    lz4_flex writes) and re-framed (header checksums by python-xxhash); then the
    batch is checked + decompressed on the device.  Random 64 B values make the
    payloads barely compressible, so this is the literal-heavy worst case."""
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
        ck = xxhash.xxh3_128_intdigest(c)
        h = b"LSM\x03\x00" + ck.to_bytes(16, "little") + len(c).to_bytes(4, "little") + \
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
    o0 = int(off[0]) + 33
    if "DIAG" not in str(lsmgpu.LIB_PATH):  # diagnostic variants (scripts/lz4_ablation.py) skip work
        assert out[:int(off[1]) - o0].cpu().numpy().tobytes() == host[o0:int(off[1])], "lz4: block 0 bytes"
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        lsmgpu.lz4_decompress_blocks(dbuf, doff)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    return {"blocks": nb, "stored_bytes": int(loff[-1]), "raw_bytes": raw_total, "ms": round(ms, 4),
            "GiB_per_s_raw": round(raw_total / (ms * 1e-3) / 2 ** 30, 1),
            "note": "header + xxh3_128 verify + LZ4 decode, wave per block; host-side size scan included"}


def load_traffic(n_blocks):
    """HBM bytes of one decode_blocks_kernel launch over n_blocks, from the
    newest committed rocprofv3 PMC summary (profiles/traffic_*.json: FETCH_SIZE
    x2 per the gfx950 guide + WRITE_SIZE), scaled per block when the profiled
    launch had a different block count."""
    best, src = None, None
    for p in sorted((ROOT / "profiles").glob("traffic_*.json")):
        try:
            best, src = json.loads(p.read_text()), p.name
        except Exception:
            pass
    if not best:
        return None, None
    return int(round(best["bytes_per_launch"] * n_blocks / best["blocks"])), f"{src} ({best['blocks']} blocks)"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--blocks", type=int, default=1 << 20)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-host", action="store_true", help="skip the host-inclusive (PCIe) measurement")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--tuning", type=str, default="", help="bpw,stage_bytes,tile_items")
    ap.add_argument("--skip-verify", action="store_true")
    ap.add_argument("--no-extra", action="store_true", help="skip the configs[3]/[4] and point-read legs")
    args = ap.parse_args()

    import torch
    import lsmgpu

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    nb = args.blocks
    tuning = tuple(int(x) for x in args.tuning.split(",")) if args.tuning else None
    check_cut_rule(lsmgpu, 52, 16, 64)
    t_gen = time.perf_counter()
    items, starts, n_items = make_workload(torch, lsmgpu, nb, seed=0x5EED0002 + rank)
    encoder = lsmgpu.Encoder(dev)
    enc = encoder.encode(items, starts, nb)
    torch.cuda.synchronize()
    total_bytes = int(enc["block_off"][nb].item())
    log(f"[rank {rank}] generated+encoded {nb} blocks, {n_items} items, {total_bytes / 2**30:.3f} GiB "
        f"in {time.perf_counter() - t_gen:.1f}s")

    dec_ctx = lsmgpu.Decoder(dev)
    item_cap = n_items
    out = dec_ctx.alloc_outputs(item_cap, nb, fields=DATA_FIELDS)
    blocks, boff = enc["buf"], enc["block_off"]

    def step(tun=tuning):
        dec_ctx.decode(blocks, boff, nb, out, item_cap, tuning=tun)

    step()
    torch.cuda.synchronize()
    checked = 0 if args.skip_verify else verify_sample(torch, lsmgpu, items, starts, enc, out, nb, n_items, rank)

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
    wall = time.perf_counter() - t0
    gpu_ms = e0.elapsed_time(e1)
    el = wall
    if dist is not None:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
        tb = torch.tensor([total_bytes], dtype=torch.int64, device=dev)
        dist.all_reduce(tb, op=dist.ReduceOp.SUM)
        all_bytes = int(tb.item())
    else:
        all_bytes = total_bytes
    ms_per_step = el * 1e3 / args.steps
    value = all_bytes * args.steps / el / 2 ** 30

    # dominant kernel alone (decode_blocks_kernel, item_start precomputed), HIP events on its stream
    base = tuning or (0, 0, 0)
    ktun = (base[0], base[1], base[2], lsmgpu.DECODE_ITEM_START_VALID)
    for _ in range(2):
        step(ktun)
    k0, k1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    k0.record()
    for _ in range(args.steps):
        step(ktun)
    k1.record()
    torch.cuda.synchronize()
    kernel_ms = k0.elapsed_time(k1) / args.steps
    alg_bytes = total_bytes + n_items * PARSED_BYTES_PER_ITEM + nb * PER_BLOCK_OUT
    achieved = alg_bytes / (kernel_ms * 1e-3) / 1e9
    traffic, traffic_src = load_traffic(nb)

    # encode (config 3 round trip) throughput on the same batch
    torch.cuda.synchronize()
    c0, c1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    esteps = max(3, args.steps // 4)
    c0.record()
    for _ in range(esteps):
        encoder.encode(items, starts, nb, out=enc)
    c1.record()
    torch.cuda.synchronize()
    enc_ms = c0.elapsed_time(c1) / esteps

    dec_ms = kernel_ms  # the decode kernel alone (item_start precomputed), for the round trip
    extra = {}
    if not args.no_extra:
        extra["point_read"] = bench_point_read(torch, lsmgpu, items, starts, enc, nb, n_items)
        extra["file_checksum"] = bench_file_checksum(torch, lsmgpu, enc, total_bytes)
        extra["bloom"] = bench_bloom(torch, lsmgpu, items, n_items)
        if rank == 0:
            extra["lz4"] = bench_lz4(torch, lsmgpu, enc, nb)
        if world == 1:
            extra["config4"] = bench_config4(torch, lsmgpu, max(3, args.steps // 4), rank)
        extra["config5"] = bench_config5(torch, lsmgpu, max(3, args.steps // 4), rank, world, dist, dev)

    hostinc = None
    if rank == 0 and world == 1 and not args.no_host:
        hostinc = host_inclusive(torch, lsmgpu, enc, out["item_start"], nb)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(torch, enc, nb, min_seconds=args.cpu_seconds)

    if rank == 0:
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
            "data": "synthetic (16 B BE-counter keys, 64 B random values, seqno 63; GPU-encoded, sample "
                    f"checked bit-exact vs oracle: {checked} blocks)",
            "config": {"workload": "BASELINE configs[1]: decode 1 M x 4 KiB data blocks, device-resident",
                       "blocks_per_gpu": nb, "items_per_gpu": n_items, "block_bytes_per_gpu": total_bytes,
                       "restart_interval": 16, "hash_ratio": 0.0, "key_len": 16, "val_len": 64,
                       "parallelism": f"shard{world} (independent block batches, no collective)",
                       "tuning": list(tuning) if tuning else "default"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBPS, 4),
                         "traffic": traffic, "traffic_source": traffic_src,
                         "kernel": "decode_blocks_kernel", "kernel_ms": round(kernel_ms, 4),
                         "alg_bytes_per_launch": alg_bytes,
                         "read_only_frac": round(total_bytes / (kernel_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4)},
            "cpu_baseline": cpu,
            "encode": {"GiB_per_s_written": round(total_bytes / (enc_ms * 1e-3) / 2 ** 30, 3),
                       "ms": round(enc_ms, 4)},
            "config3_roundtrip": {"workload": "BASELINE configs[2]: encode + checksum + decode of the same batch, "
                                              "bit-exact block bytes vs the oracle (sampled)",
                                  "encode_ms": round(enc_ms, 4), "decode_ms": round(dec_ms, 4),
                                  "GiB_per_s": round(total_bytes / ((enc_ms + dec_ms) * 1e-3) / 2 ** 30, 3)},
            **extra,
            "host_inclusive_decode": hostinc,
            "gpu_event_ms_per_step": round(gpu_ms / args.steps, 4),
        }
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
