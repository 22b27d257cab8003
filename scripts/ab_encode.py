#!/usr/bin/env python3
"""A/B timing of library variants on the encode (and decode) bench workloads.

usage: scripts/ab_encode.py LIB1 LIB2 ... [--rounds 3]
Each round runs every library in its own child process (interleaved, rule 24 of
the HIP guide); a child times lsm_encode_blocks on configs[1] (1 M x 4 KiB) and
configs[3] (256 K x 16 KiB prefix keys) and prints the xxh3_128 of the encoded
bytes, so variants can be compared for identical output.
"""
import json
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def child(reps, which):
    for p in (ROOT, ROOT / "lsm-tree_amd", ROOT / "oracle", ROOT / "tests"):
        sys.path.insert(0, str(p))
    import torch
    import bench
    import lsmgpu
    torch.cuda.set_device(0)
    res = {}
    shapes = {"c1": dict(n_blocks=1 << 20), "c3": dict(n_blocks=262144, items_per_block=56, key_len=40, val_len=256,
                                                      kind="prefix"),
              "r1": dict(n_blocks=1 << 20, kind="random"),
              "h1": dict(n_blocks=1 << 20),  # configs[1] with the hash index (ratio 1.33, bench_hash_index)
              # the configs[4] data-block classes (bench.C5_SEGMENTS, ~1.4 GB each)
              "k16c": dict(n_blocks=97817, items_per_block=205), "k16r": dict(n_blocks=82754, items_per_block=205,
                                                                           kind="random"),
              "k64c": dict(n_blocks=24552, items_per_block=820), "k64r": dict(n_blocks=20682, items_per_block=820,
                                                                           kind="random"),
              # the large-block legs (bench_large_blocks: the writer's 1 / 4 MiB data blocks, the workspace pool)
              "l1m": dict(n_blocks=240, items_per_block=13108, seed=0x5EED0007),
              "l4m": dict(n_blocks=60, items_per_block=52429, seed=0x5EED0007)}
    for name in which.split(","):
        off32 = name.endswith("_32")  # the same shape through lsm_encode_blocks32 (u32 offsets)
        base = name[:-3] if off32 else name
        items, starts, n = bench.make_workload(torch, lsmgpu, **shapes[base])
        if off32:
            items = dict(items, key_off=items["key_off"].to(torch.int32), val_off=items["val_off"].to(torch.int32))
        nb = shapes[base]["n_blocks"]
        hr = 1.33 if base == "h1" else 0.0
        enc_ctx = lsmgpu.Encoder()
        enc = enc_ctx.encode(items, starts, nb, hash_ratio=hr)
        torch.cuda.synchronize()
        total = int(enc["block_off"][nb].item())
        bad = int((enc["status"][:nb] != 0).sum())
        # untimed warm-up calls: without them the first shape of a child ran ~3-5 % slow
        # (clocks / allocator still settling), which biased cross-shape comparisons
        for _ in range(5):
            enc_ctx.encode(items, starts, nb, hash_ratio=hr, out=enc)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            enc_ctx.encode(items, starts, nb, hash_ratio=hr, out=enc)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        ck = lsmgpu.xxh3_128_file(enc["buf"], total)
        res[name] = {"ms": round(ms, 4), "bytes": total, "bad": bad, "ck": f"{ck[1]:016x}{ck[0]:016x}"}
        del items, enc
        torch.cuda.empty_cache()
    print(json.dumps(res), flush=True)


def main():
    if sys.argv[1] == "--child":
        child(int(sys.argv[2]), sys.argv[3])
        return
    libs, rounds, which, reps = [], 3, "c1,c3", 10
    a = sys.argv[1:]
    while a:
        x = a.pop(0)
        if x == "--rounds":
            rounds = int(a.pop(0))
        elif x == "--which":
            which = a.pop(0)
        elif x == "--reps":
            reps = int(a.pop(0))
        else:
            libs.append(x)
    out = {l: [] for l in libs}
    for r in range(rounds):
        for l in libs:
            env = dict(os.environ, LSMGPU_LIB=str(Path(l).resolve()))
            p = subprocess.run([sys.executable, __file__, "--child", str(reps), which], env=env, capture_output=True,
                               text=True, timeout=300)
            if p.returncode != 0:
                print(l, "FAILED", p.stderr[-2000:], flush=True)
                sys.exit(p.returncode)
            d = json.loads(p.stdout.strip().splitlines()[-1])
            out[l].append(d)
            print(f"round {r} {Path(l).name:28s} " + "  ".join(f"{k} {v['ms']:.4f} ms bad {v['bad']} ck {v['ck'][:12]}"
                                                          for k, v in d.items()), flush=True)
    print("median:")
    for l in libs:
        ks = out[l][0].keys()
        print(f"  {Path(l).name:28s} " + "  ".join(
            f"{k} {sorted(x[k]['ms'] for x in out[l])[len(out[l]) // 2]:.4f} ms" for k in ks))


if __name__ == "__main__":
    main()
