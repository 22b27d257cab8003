#!/usr/bin/env python3
"""Experiment (verdict r05 item 1): does encoding configs[1] in sub-batches whose plan input fits
the 256 MB MALL beat one call?  Each sub-batch is one lsm_encode_blocks32 call over a slice of
the block starts (absolute item indices), so the group kernel of a chunk re-reads item fields
and keys the chunk's plan kernel read just before.  Times one whole call against back-to-back
chunk calls (one output buffer and workspace, reused) for several chunk sizes.

usage: python scripts/exp/enc_chunked.py [--reps 5] [--chunks 32768,65536,131072,262144]"""
import ctypes as C
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
for p in (ROOT, ROOT / "lsm-tree_amd"):
    sys.path.insert(0, str(p))


def main():
    import torch
    import bench
    import lsmgpu
    reps, chunks = 5, [32768, 65536, 131072, 262144]
    a = sys.argv[1:]
    while a:
        x = a.pop(0)
        if x == "--reps":
            reps = int(a.pop(0))
        elif x == "--chunks":
            chunks = [int(v) for v in a.pop(0).split(",")]
    torch.cuda.set_device(0)
    nb = 1 << 20
    items, starts, _ = bench.make_workload(torch, lsmgpu, n_blocks=nb)
    items = dict(items, key_off=items["key_off"].to(torch.int32), val_off=items["val_off"].to(torch.int32))
    enc = lsmgpu.Encoder()
    out = enc.encode(items, starts, nb)
    torch.cuda.synchronize()
    lib = lsmgpu.lib()
    it = lsmgpu.LsmItems32()
    it.keys, it.key_off = items["keys"].data_ptr(), items["key_off"].data_ptr()
    it.vals, it.val_off = items["vals"].data_ptr(), items["val_off"].data_ptr()
    it.seqno, it.vtype = items["seqno"].data_ptr(), items["vtype"].data_ptr()
    it.n_items = items["seqno"].numel()
    params = lsmgpu.LsmBlockParams(16, 0, 0, 0, 0.0, 0)
    cap = out["buf"].numel() - lsmgpu.LSM_INPUT_PADDING
    ws = enc.ws
    stream = C.c_void_p(torch.cuda.current_stream().cuda_stream)

    def call(b0, n):
        rc = lib.lsm_encode_blocks32(C.byref(it), C.c_void_p(starts.data_ptr() + 4 * b0), n, C.byref(params),
                                     C.c_void_p(out["buf"].data_ptr()), cap,
                                     C.c_void_p(out["block_off"].data_ptr() + 8 * b0),
                                     C.c_void_p(out["status"].data_ptr() + 4 * b0),
                                     C.c_void_p(ws.data_ptr()), ws.numel(), stream)
        assert rc == 0, rc

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps

    res = {"whole": round(timed(lambda: call(0, nb)), 4)}
    for c in chunks:
        def run(c=c):
            for b0 in range(0, nb, c):
                call(b0, min(c, nb - b0))
        res[str(c)] = round(timed(run), 4)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
