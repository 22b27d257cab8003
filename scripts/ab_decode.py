#!/usr/bin/env python3
"""A/B timing of library variants on the decode bench workloads.

usage: scripts/ab_decode.py LIB1 LIB2 ... [--rounds 3] [--which c1,c3] [--modes full,compact,call]
(modes full / compact: the decode with item_start precomputed; call: the whole lsm_decode_blocks call)
Each round runs every library in its own child process (interleaved); a child
encodes the workload once, then times lsm_decode_blocks (item_start
precomputed) in each output mode, interleaved within the child as well, and
prints a checksum of the parsed fields so variants can be compared for
identical output.
"""
import json
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def child(reps, which, modes):
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
              # the configs[4] size classes (1.4 GB each, bench.C5_SEGMENTS)
              "k16c": dict(n_blocks=97817, items_per_block=205), "k16r": dict(n_blocks=82754, items_per_block=205,
                                                                           kind="random"),
              "k64c": dict(n_blocks=24552, items_per_block=820), "k64r": dict(n_blocks=20682, items_per_block=820,
                                                                           kind="random")}
    for name in which.split(","):
        items, starts, n = bench.make_workload(torch, lsmgpu, **shapes[name])
        nb = shapes[name]["n_blocks"]
        enc = lsmgpu.Encoder().encode(items, starts, nb)
        torch.cuda.synchronize()
        del items
        dec = lsmgpu.Decoder()
        outs = {m: dec.alloc_outputs(n, nb, fields=None if m == "compact" else bench.DATA_FIELDS,
                                     compact=m == "compact") for m in modes}
        tune = (0, 0, 0, lsmgpu.DECODE_ITEM_START_VALID)
        for m in modes:
            dec.decode(enc["buf"], enc["block_off"], nb, outs[m], n, compact=m == "compact")
        torch.cuda.synchronize()
        times = {m: [] for m in modes}
        for _ in range(3):
            for m in modes:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(reps):  # (mode "call": the whole call, item_start counted and scanned too)
                    dec.decode(enc["buf"], enc["block_off"], nb, outs[m], n, tuning=None if m == "call" else tune,
                               compact=m == "compact")
                e1.record()
                torch.cuda.synchronize()
                times[m].append(e0.elapsed_time(e1) / reps)
        for m in modes:
            o = outs[m]
            bad = int((o["status"][:nb] != 0).sum())
            ck = int(sum(int(o[f][:n].to(torch.int64).sum()) for f in ("key_off", "val_off", "val_len", "key_len")))
            ck += int(o["item_start"][:nb + 1].to(torch.int64).sum())
            res[f"{name}.{m}"] = {"ms": round(min(times[m]), 4), "bad": bad, "ck": ck}
        del enc, outs
        torch.cuda.empty_cache()
    print(json.dumps(res), flush=True)


def main():
    if sys.argv[1] == "--child":
        child(int(sys.argv[2]), sys.argv[3], sys.argv[4].split(","))
        return
    libs, rounds, which, reps, modes = [], 3, "c1", 10, "full,compact"
    a = sys.argv[1:]
    while a:
        x = a.pop(0)
        if x == "--rounds":
            rounds = int(a.pop(0))
        elif x == "--which":
            which = a.pop(0)
        elif x == "--reps":
            reps = int(a.pop(0))
        elif x == "--modes":
            modes = a.pop(0)
        else:
            libs.append(x)
    out = {l: [] for l in libs}
    for r in range(rounds):
        for l in libs:
            env = dict(os.environ, LSMGPU_LIB=str(Path(l).resolve()))
            p = subprocess.run([sys.executable, __file__, "--child", str(reps), which, modes], env=env,
                               capture_output=True, text=True, timeout=300)
            if p.returncode != 0:
                print(l, "FAILED", p.stderr[-2000:], flush=True)
                sys.exit(p.returncode)
            d = json.loads(p.stdout.strip().splitlines()[-1])
            out[l].append(d)
            print(f"round {r} {Path(l).name:28s} " + "  ".join(f"{k} {v['ms']:.4f} ms bad {v['bad']} ck {v['ck']}"
                                                          for k, v in d.items()), flush=True)
    print("median:")
    for l in libs:
        ks = out[l][0].keys()
        print(f"  {Path(l).name:28s} " + "  ".join(
            f"{k} {sorted(x[k]['ms'] for x in out[l])[len(out[l]) // 2]:.4f} ms" for k in ks))


if __name__ == "__main__":
    main()
