#!/usr/bin/env python3
"""Per-kernel mean of every PMC counter found under rocprofv3 output dirs.
usage: pmc_table.py KERNEL_SUBSTR DIR [DIR ...]"""
import csv
import glob
import os
import sys
from collections import defaultdict

kern = sys.argv[1]
vals = defaultdict(list)
meta = {}
for d in sys.argv[2:]:
    files = [d] if os.path.isfile(d) else glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if kern in row["Kernel_Name"]:
                    vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
                    meta = {k: row[k] for k in ("Kernel_Name", "VGPR_Count", "Scratch_Size", "LDS_Block_Size", "Grid_Size")}
print(meta)
for k in sorted(vals):
    v = vals[k]
    print(f"{k:32s} {sum(v) / len(v):16.1f}  (n={len(v)})")
