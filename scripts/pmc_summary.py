#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSV passes of scripts/prof_decode.py per variant."""
import csv
import json
import sys
from collections import defaultdict
from pathlib import Path

VARIANTS = ["full", "no-parse", "stage-only", "no-hash", "phaseA-only"]


def load(dirpath):
    rows = []
    for f in Path(dirpath).rglob("*counter_collection.csv"):
        with open(f) as fh:
            rows.extend(csv.DictReader(fh))
    return rows


def main():
    root = Path(sys.argv[1])
    per = defaultdict(lambda: defaultdict(float))  # (variant) -> counter -> value (mean over reps)
    counts = defaultdict(lambda: defaultdict(int))
    for pdir in sorted(root.glob("p*")):
        if not pdir.is_dir():
            continue
        rows = [r for r in load(pdir) if ("decode_blocks_kernel" in r.get("Kernel_Name", "") or "decode_ring_kernel" in r.get("Kernel_Name", ""))]
        by_disp = defaultdict(lambda: defaultdict(float))
        for r in rows:
            by_disp[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
        disp = sorted(by_disp)
        disp = disp[1:]  # first dispatch = warm-up decode (full, computes item_start)
        for idx, d in enumerate(disp):
            v = VARIANTS[idx % len(VARIANTS)]
            for c, val in by_disp[d].items():
                per[v][c] += val
                counts[v][c] += 1
    out = {}
    for v in VARIANTS:
        out[v] = {c: per[v][c] / counts[v][c] for c in sorted(per[v])}
    print(json.dumps(out, indent=1))
    if "full" in out and "SQ_INSTS_VALU" in out["full"]:
        f, s = out["full"], out.get("stage-only", {})
        print("\nper-wave-instruction deltas (full - stage-only):")
        for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_WAVE_CYCLES", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "SQ_BUSY_CYCLES", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_LDS_BANK_CONFLICT", "SQ_WAIT_INST_LDS"):
            if c in f:
                print(f"  {c:22s} full {f[c]:14.0f}  stage-only {s.get(c, 0):14.0f}  delta {f[c] - s.get(c, 0):14.0f}")


if __name__ == "__main__":
    main()
