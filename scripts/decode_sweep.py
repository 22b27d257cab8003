#!/usr/bin/env python3
"""Decode tuning sweep + phase ablations on the bench workload (diagnostic).

Times decode_blocks_kernel alone (item_start precomputed) for several
(blocks_per_wave, stage_bytes, tile_items) tunings, and prices each phase by
dropping it (diagnostic flags; outputs invalid in those runs).  Interleaved
rounds in one process (cdna_hip_programming.md §5.4 rule 24).
"""
import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
for p in (ROOT, ROOT / "lsm-tree_amd", ROOT / "oracle", ROOT / "tests"):
    sys.path.insert(0, str(p))

import torch  # noqa: E402

import bench  # noqa: E402
import lsmgpu  # noqa: E402

SKIP_HASH, SKIP_PARSE, SKIP_STORE = 0x100, 0x200, 0x400


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", type=int, default=1 << 20)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--tunings", default="48,65536,1024,0x10000;0,32768,512;0,32768,512,0x20000")
    ap.add_argument("--ablate", default="0,32768,512")
    ap.add_argument("--workload", default="counter", choices=["counter", "prefix16k"])
    args = ap.parse_args()
    torch.cuda.set_device(0)
    nb = args.blocks
    if args.workload == "counter":
        items, starts, n_items = bench.make_workload(torch, lsmgpu, nb)
    else:
        items, starts, n_items = bench.make_workload(torch, lsmgpu, nb, items_per_block=56, key_len=40, val_len=256)
    enc = lsmgpu.Encoder().encode(items, starts, nb)
    torch.cuda.synchronize()
    total = int(enc["block_off"][nb].item())
    dec = lsmgpu.Decoder()
    out = dec.alloc_outputs(n_items, nb)
    dec.decode(enc["buf"], enc["block_off"], nb, out, n_items)
    torch.cuda.synchronize()
    assert int((out["status"][:nb] != 0).sum()) == 0

    variants = {}
    def tun(v, extra=0):
        v = list(v) + [0] * (4 - len(v))
        v[3] |= 1 | extra
        return tuple(v)

    for t in args.tunings.replace("/", ";").split(";"):
        variants[f"tune {t}"] = tun([int(x, 0) for x in t.split(",")])
    if args.ablate:
        a = [int(x, 0) for x in args.ablate.split(",")]
        variants["ablate no-hash"] = tun(a, SKIP_HASH)
        variants["ablate no-parse"] = tun(a, SKIP_PARSE)
        variants["ablate no-store"] = tun(a, SKIP_STORE)
        variants["ablate phase-A only"] = tun(a, 0x800)
        variants["ablate A no-hash"] = tun(a, 0x800 | SKIP_HASH)
        variants["ablate stage-only"] = tun(a, SKIP_HASH | SKIP_PARSE | SKIP_STORE)
    times = {k: [] for k in variants}
    for _ in range(args.rounds):
        for name, tun in variants.items():
            dec.decode(enc["buf"], enc["block_off"], nb, out, n_items, tuning=tun)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.reps):
                dec.decode(enc["buf"], enc["block_off"], nb, out, n_items, tuning=tun)
            e1.record()
            torch.cuda.synchronize()
            times[name].append(e0.elapsed_time(e1) / args.reps)
    alg = total + n_items * bench.PARSED_BYTES_PER_ITEM + nb * bench.PER_BLOCK_OUT
    res = []
    for name, ts in times.items():
        ms = min(ts)
        res.append({"variant": name, "ms_min": round(ms, 4), "ms_all": [round(x, 4) for x in ts],
                    "GBps_alg": round(alg / ms / 1e6, 1), "GiBps_read": round(total / ms * 1e3 / 2 ** 30, 1)})
        print(f"{name:28s} {ms:8.4f} ms  {alg / ms / 1e6:8.1f} GB/s alg  {total / ms * 1e3 / 2**30:8.1f} GiB/s in",
              flush=True)
    print(json.dumps({"workload": args.workload, "blocks": nb, "bytes": total, "items": n_items, "results": res}))


if __name__ == "__main__":
    main()
