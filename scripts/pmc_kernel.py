#!/usr/bin/env python3
"""Per-dispatch mean of rocprofv3 --pmc counters for one kernel, per block
(diagnostic): python scripts/pmc_kernel.py DIR KERNEL_SUBSTRING N_BLOCKS."""
import csv
import sys
from collections import defaultdict
from pathlib import Path

root, name, nb = Path(sys.argv[1]), sys.argv[2], int(sys.argv[3])
by = defaultdict(lambda: defaultdict(float))
for f in root.rglob("*counter_collection.csv"):
    with open(f) as fh:
        for r in csv.DictReader(fh):
            if name in r.get("Kernel_Name", ""):
                by[(str(f), int(r["Dispatch_Id"]))][r["Counter_Name"]] += float(r["Counter_Value"])
acc = defaultdict(list)
for d in by.values():
    for c, v in d.items():
        acc[c].append(v)
for c in sorted(acc):
    v = sum(acc[c]) / len(acc[c])
    print(f"{c:24s} per dispatch {v:16.0f}   per block {v / nb:12.2f}")
