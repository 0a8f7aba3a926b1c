#!/usr/bin/env python3
"""Per-kernel PMC summary of ``scripts/gpu_pmc_step.sh`` (rocprofv3 CSV counter collection).

Per kernel (summed over dispatches): time, MFMA instructions -> delivered TFLOP/s
(16x16x32 bf16/f16 MFMA = 16,384 FLOP per wave instruction) and its share of the 2.5 PFLOP/s
dense bf16 peak, LDS bank-conflict ratio
(SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE) and HBM read bandwidth from FETCH_SIZE
(KiB, doubled: gfx950 tallies a wide coalesced read at half its bytes,
MI355X_MICROARCH.md "FETCH_SIZE"). Durations are from counter-collection dispatches, which
run serialised, so they are slightly longer than in the graph-launched step.

usage: pmc_summary.py <pass1 counter_collection.csv> [<pass2 counter_collection.csv>] [--top N]
"""
from __future__ import annotations

import csv
import sys
from collections import defaultdict

FLOP_PER_MFMA = 16 * 16 * 32 * 2
PEAK_TFLOPS = 2500.0


def load(path):
    disp = {}
    for row in csv.DictReader(open(path)):
        key = row["Dispatch_Id"]
        d = disp.setdefault(key, {"name": row["Kernel_Name"], "t": int(row["End_Timestamp"]) - int(row["Start_Timestamp"])})
        d[row["Counter_Name"]] = d.get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
    return disp


def short(name: str) -> str:
    name = name.replace("void ", "")
    return name.split("(")[0][:70]


def main(argv):
    top = 25
    if "--top" in argv:
        i = argv.index("--top")
        top = int(argv[i + 1])
        argv = argv[:i] + argv[i + 2:]
    agg = defaultdict(lambda: defaultdict(float))
    for path in argv:
        for d in load(path).values():
            a = agg[short(d["name"])]
            a["n_" + path] += 1
            a["t_" + path] += d["t"]
            for k, v in d.items():
                if k not in ("name", "t"):
                    a[k] += v
    p1 = argv[0]
    rows = sorted(agg.items(), key=lambda kv: -kv[1]["t_" + p1])
    tot_t = sum(a["t_" + p1] for _, a in rows)
    tot_mfma = sum(a["SQ_INSTS_MFMA"] for _, a in rows)
    print("%-70s %5s %9s %6s %8s %6s %6s %8s" % ("kernel", "n", "us", "share", "TFLOP/s", "%peak", "ldsbc", "rd GB/s"))
    for name, a in rows[:top]:
        t = a["t_" + p1]
        tf = a["SQ_INSTS_MFMA"] * FLOP_PER_MFMA / t / 1e3 if t else 0.0
        busy = tf / PEAK_TFLOPS
        bc = a["SQ_LDS_BANK_CONFLICT"] / a["SQ_LDS_IDX_ACTIVE"] if a["SQ_LDS_IDX_ACTIVE"] else 0.0
        rd = ""
        if len(argv) > 1 and a["t_" + argv[1]]:
            rd = "%.0f" % (a["FETCH_SIZE"] * 1024 * 2 / a["t_" + argv[1]])
        print("%-70s %5d %9.1f %5.1f%% %8.1f %5.1f%% %6.3f %8s" % (
            name, a["n_" + p1], t / 1e3, 100 * t / tot_t, tf, 100 * busy, bc, rd))
    print("\nall kernels: %.1f us, MFMA work %.1f GFLOP -> %.1f TFLOP/s averaged over kernel time"
          % (tot_t / 1e3, tot_mfma * FLOP_PER_MFMA / 1e9, tot_mfma * FLOP_PER_MFMA / tot_t / 1e3))


if __name__ == "__main__":
    main(sys.argv[1:])
