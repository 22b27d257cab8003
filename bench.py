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


def make_workload(torch, lsmgpu, n_blocks, items_per_block=52, key_len=16, val_len=64, seed=0x5EED0002):
    dev = "cuda"
    n = n_blocks * items_per_block
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    ctr = torch.arange(n, dtype=torch.int64, device=dev)
    keys = torch.zeros(n * key_len + lsmgpu.LSM_INPUT_PADDING, dtype=torch.uint8, device=dev)
    kv = keys[:n * key_len].view(n, key_len)
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


def check_cut_rule(lsmgpu, items_per_block, key_len, val_len):
    """The fixed 52-item cut equals the reference writer rule (writer/mod.rs:284-290)."""
    import numpy as np
    m = items_per_block * 4
    ko = np.arange(m + 1, dtype=np.uint64) * key_len
    vo = np.arange(m + 1, dtype=np.uint64) * val_len
    starts = lsmgpu.cut_blocks(ko, vo, 4096)
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


def load_traffic():
    """HBM bytes per decode launch from the committed rocprofv3 PMC summary
    (profiles/traffic_*.json), FETCH_SIZE doubled per the gfx950 guide."""
    best = None
    for p in sorted((ROOT / "profiles").glob("traffic_*.json")):
        try:
            best = json.loads(p.read_text())
        except Exception:
            pass
    return best


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
    traffic = load_traffic()

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
                         "traffic": traffic.get("bytes_per_launch") if traffic else None,
                         "kernel": "decode_blocks_kernel", "kernel_ms": round(kernel_ms, 4),
                         "alg_bytes_per_launch": alg_bytes,
                         "read_only_frac": round(total_bytes / (kernel_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4)},
            "cpu_baseline": cpu,
            "encode": {"GiB_per_s_written": round(total_bytes / (enc_ms * 1e-3) / 2 ** 30, 3),
                       "ms": round(enc_ms, 4)},
            "host_inclusive_decode": hostinc,
            "gpu_event_ms_per_step": round(gpu_ms / args.steps, 4),
        }
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
