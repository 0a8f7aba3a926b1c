#!/usr/bin/env python3
"""Per-kernel mean of every collected PMC counter per dispatch (rocprofv3 CSV), plus derived
cycles: SQ_WAVE_CYCLES / SQ_BUSY_CYCLES etc. are quad-cycles (x4), SQ_VALU_MFMA_BUSY_CYCLES cycles.
usage: pmc_kernel.py <counter_collection.csv> [...]"""
import csv
import sys
from collections import defaultdict

for path in sys.argv[1:]:
    disp = {}
    for row in csv.DictReader(open(path)):
        d = disp.setdefault(row["Dispatch_Id"], {"name": row["Kernel_Name"].split("(")[0][:60],
                                                 "t": int(row["End_Timestamp"]) - int(row["Start_Timestamp"])})
        d[row["Counter_Name"]] = d.get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
    by = defaultdict(list)
    for d in disp.values():
        by[d["name"]].append(d)
    for name, ds in by.items():
        keys = sorted(k for k in ds[0] if k not in ("name", "t"))
        print("%s  (%d dispatches, mean %.1f us)" % (name, len(ds), sum(d["t"] for d in ds) / len(ds) / 1e3))
        for k in keys:
            print("   %-28s %16.0f" % (k, sum(d.get(k, 0) for d in ds) / len(ds)))
