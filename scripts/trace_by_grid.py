#!/usr/bin/env python3
"""Per-(kernel, grid) duration summary of a rocprofv3 --kernel-trace CSV, lsmgpu
kernels only: the bench launches the decode kernel over several batches
(configs[1], [3], [4]), and each batch has its own grid, so the configs[1]
launches are the rows with its grid.  usage: trace_by_grid.py TRACE.csv > OUT.csv"""
import csv
import sys
from collections import defaultdict

rows = defaultdict(list)
with open(sys.argv[1]) as fh:
    for r in csv.DictReader(fh):
        name = r["Kernel_Name"]
        if "lsmgpu::" not in name:
            continue
        grid = int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))
        rows[(name.split("(")[0].replace("void ", "").replace("lsmgpu::", ""), grid)].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
w = csv.writer(sys.stdout)
w.writerow(["kernel", "workgroups", "calls", "avg_us", "min_us", "max_us"])
for (k, g), d in sorted(rows.items(), key=lambda kv: -sum(kv[1])):
    w.writerow([k, g, len(d), round(sum(d) / len(d) / 1e3, 1), round(min(d) / 1e3, 1), round(max(d) / 1e3, 1)])
