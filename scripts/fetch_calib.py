#!/usr/bin/env python3
"""FETCH_SIZE / WRITE_SIZE calibration of the encode kernels' access shapes
(measurement only; verdict r04 item 4).

The guide calibrates FETCH_SIZE only for 16 B/lane streams (it reads half the
bytes).  Here every shape the encode kernels use touches a known number of
bytes of a buffer far larger than the 256 MiB Infinity Cache, once per
dispatch (lsm_ceiling_fetch_calib in lsm-tree_amd/ceiling/ceiling.hip):

  python scripts/fetch_calib.py run                     # the dispatches (under rocprofv3)
  python scripts/fetch_calib.py summary PMC_DIR PMC_DIR # factor = bytes / counter bytes

Every mode is dispatched REPS times in MODES order; the summary maps dispatch
order back to modes."""
import ctypes as C
import csv
import json
import sys
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
# mode -> (element bytes, threads per element, what it stands for, read or write)
MODES = {0: (8, "u64 lane-contiguous (E2 item fields)", "r"),
         1: (8, "u64, lane t: 2t..2t+2 (E1 key / value offsets)", "r"),
         2: (8, "u64, lane t: 2t, 2t+1 (E1 seqnos)", "r"),
         3: (1, "u8, lane t: 2t, 2t+1 (E1 value types)", "r"),
         4: (1, "u8 lane-contiguous (E2 value types)", "r"),
         5: (4, "u32 lane-contiguous (E2 erec)", "r"),
         6: (16, "16 B lane-contiguous (the guide's calibrated shape)", "r"),
         7: (4, "u32 stores, lane t: 2t, 2t+1 (E1 erec)", "w"),
         8: (4, "u32 stores lane-contiguous", "w")}
BYTES = 2 << 30  # per mode: 8x the Infinity Cache
REPS = 2


def run():
    import torch
    lib = C.CDLL(str(ROOT / "lsm-tree_amd" / "ceiling" / "liblsmceiling.so"))
    lib.lsm_ceiling_fetch_calib.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_int, C.c_void_p, C.c_void_p]
    buf = torch.randint(0, 256, (BYTES + 64,), dtype=torch.uint8, device="cuda")
    wbuf = torch.empty(BYTES + 64, dtype=torch.uint8, device="cuda")
    sink = torch.zeros(4, dtype=torch.int32, device="cuda")
    s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    for mode, (esz, what, rw) in MODES.items():
        n = BYTES // esz
        for _ in range(REPS):
            assert lib.lsm_ceiling_fetch_calib(buf.data_ptr(), wbuf.data_ptr(), n, mode, sink.data_ptr(), s) == 0
        torch.cuda.synchronize()
        print(f"mode {mode}: {n} x {esz} B ({what})", flush=True)


def summary(dirs):
    vals = defaultdict(lambda: defaultdict(float))  # counter -> dispatch -> value
    for d in dirs:
        for f in Path(d).rglob("*counter_collection.csv"):
            with open(f) as fh:
                for r in csv.DictReader(fh):
                    if "fetch_calib_kernel" in r.get("Kernel_Name", ""):
                        vals[r["Counter_Name"]][int(r["Dispatch_Id"])] += float(r["Counter_Value"])
    out = {}
    for counter, by in vals.items():
        ids = sorted(by)
        assert len(ids) == REPS * len(MODES), (counter, len(ids))
        for k, (mode, (esz, what, rw)) in enumerate(MODES.items()):
            kb = sum(by[i] for i in ids[REPS * k:REPS * (k + 1)]) / REPS
            e = out.setdefault(str(mode), {"shape": what, "bytes": BYTES, "dir": rw})
            e[counter + "_kb"] = round(kb, 1)
            e[counter + "_factor"] = round(BYTES / (kb * 1024), 4) if kb else None
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run()
    else:
        summary(sys.argv[2:])
