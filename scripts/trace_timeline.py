#!/usr/bin/env python3
"""Dispatch timeline from a rocprofv3 kernel trace: one line per dispatch in
start order (kernel, workgroups, duration, gap after the previous dispatch's
end), for reading where a short multi-kernel call spends its time.
usage: trace_timeline.py TRACE_DIR [--last N] [--match SUBSTR]"""
import argparse
import csv
from pathlib import Path


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--last", type=int, default=60)
    ap.add_argument("--match", default="")
    a = ap.parse_args()
    rows = []
    for f in Path(a.dir).rglob("*kernel_trace.csv"):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                name = r["Kernel_Name"].replace("lsmgpu::", "")
                name = name.split("(")[0] if "(" in name and "<" not in name.split("(")[0] else name[:70]
                wg = int(r.get("Grid_Size_X", r.get("Grid_Size", 0)) or 0) // max(1, int(r.get("Workgroup_Size_X", r.get("Workgroup_Size", 1)) or 1))
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name, wg))
    rows.sort()
    if a.match:
        rows = [r for r in rows if a.match in r[2]] if not a.match.startswith("after:") else rows
    rows = rows[-a.last:]
    prev = None
    for s, e, name, wg in rows:
        gap = (s - prev) / 1000 if prev is not None else 0.0
        print(f"{(e - s) / 1000:9.1f} us  gap {gap:7.1f}  wg {wg:6d}  {name}")
        prev = e


if __name__ == "__main__":
    main()
