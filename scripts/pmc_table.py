#!/usr/bin/env python3
"""Per-block view of a pmc_summary.py JSON (diagnostic): python scripts/pmc_table.py FILE [BLOCKS]."""
import json
import sys

t = open(sys.argv[1]).read()
j = json.loads(t[:t.index("\nper-wave")] if "\nper-wave" in t else t)
nb = int(sys.argv[2]) if len(sys.argv) > 2 else 262144
keys = ["SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
        "SQ_LDS_BANK_CONFLICT", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "FETCH_SIZE", "WRITE_SIZE",
        "GRBM_GUI_ACTIVE", "SQ_BUSY_CYCLES"]
print("%-14s" % "per block" + "".join("%11s" % k[3:13] for k in keys))
for v, d in j.items():
    print("%-14s" % v + "".join("%11.1f" % (d.get(k, 0) / nb) for k in keys))
