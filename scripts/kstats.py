#!/usr/bin/env python3
"""Print name / calls / average us of the lsmgpu kernels in rocprofv3
--stats CSVs (diagnostic): python scripts/kstats.py DIR [DIR ...]."""
import csv
import sys
from pathlib import Path

for d in sys.argv[1:]:
    for f in sorted(Path(d).rglob("*kernel_stats.csv")):
        print(f"== {f.parent}")
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if "lsmgpu" in r["Name"] or "ceiling" in r["Name"] or "copy_tile" in r["Name"]:
                    name = r["Name"].split("(")[0].replace("lsmgpu::", "")
                    print(f"  {name:60s} {int(r['Calls']):5d} {float(r['AverageNs']) / 1e3:10.1f} us")
