#!/usr/bin/env python3
"""Per-kernel PMC summary of scripts/gpu_prof_r2.sh (two rocprofv3 counter passes over eager
training steps). Per kernel, summed over dispatches:
  TFLOP/s   SQ_INSTS_MFMA x 16,384 FLOP (16x16x32 bf16) / dispatch time; %peak of 2.5 PFLOP/s
  VALU:MFMA SQ_INSTS_VALU / SQ_INSTS_MFMA (on CDNA SQ_INSTS_VALU also counts the MFMAs, so the
            non-MFMA VALU ratio is (VALU - MFMA) / MFMA, printed as "valu/mf")
  lds/mf    SQ_INSTS_LDS per MFMA; ldsbc = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
  wait%     SQ_WAIT_ANY / SQ_WAVE_CYCLES (parked on s_waitcnt / barrier), stall% = SQ_WAIT_INST_ANY
            / SQ_WAVE_CYCLES (issue stalls), active% = SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES (pass 2)
  rd GB/s   FETCH_SIZE (KiB, x2: gfx950 tallies wide coalesced reads at half) / dispatch time (pass 2)
usage: pmc_summary2.py <pass1 counter_collection.csv> <pass2 counter_collection.csv> [--top N] [--steps S]
"""
import csv
import sys
from collections import defaultdict

FLOP = 16 * 16 * 32 * 2


def load(path):
    disp = {}
    for row in csv.DictReader(open(path)):
        d = disp.setdefault(row["Dispatch_Id"], {"name": row["Kernel_Name"],
                                                 "t": int(row["End_Timestamp"]) - int(row["Start_Timestamp"])})
        d[row["Counter_Name"]] = d.get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
    return disp


def short(n):
    return n.replace("void ", "").split("(")[0][:64]


def agg(path):
    a = defaultdict(lambda: defaultdict(float))
    for d in load(path).values():
        if "dcg" not in d["name"]:
            continue
        k = a[short(d["name"])]
        k["n"] += 1
        k["t"] += d["t"]
        for c, v in d.items():
            if c not in ("name", "t"):
                k[c] += v
    return a


def main(argv):
    top = 40
    if "--top" in argv:
        i = argv.index("--top"); top = int(argv[i + 1]); argv = argv[:i] + argv[i + 2:]
    a1, a2 = agg(argv[0]), agg(argv[1])
    rows = sorted(a1.items(), key=lambda kv: -kv[1]["t"])
    tt = sum(v["t"] for _, v in rows)
    print("%-64s %4s %8s %5s %7s %5s %7s %6s %6s %5s %5s %5s %7s" % (
        "kernel", "n", "us", "share", "TFLOP/s", "%pk", "valu/mf", "lds/mf", "ldsbc", "wait", "stall", "activ", "rdGB/s"))
    for name, v in rows[:top]:
        mf = v["SQ_INSTS_MFMA"]
        tf = mf * FLOP / v["t"] / 1e3 if v["t"] else 0
        wc = v["SQ_WAVE_CYCLES"] or 1
        b = a2.get(name, {})
        wc2 = b.get("SQ_WAVE_CYCLES", 0) or wc
        rd = b.get("FETCH_SIZE", 0) * 2048 / b["t"] if b and b.get("t") else 0
        print("%-64s %4d %8.1f %4.1f%% %7.1f %4.1f%% %7s %6s %6.3f %4.0f%% %4.0f%% %4.0f%% %7.0f" % (
            name, v["n"], v["t"] / 1e3, 100 * v["t"] / tt, tf, tf / 25,
            ("%.2f" % ((v["SQ_INSTS_VALU"] - mf) / mf)) if mf else "-",
            ("%.2f" % (v["SQ_INSTS_LDS"] / mf)) if mf else "-",
            v["SQ_LDS_BANK_CONFLICT"] / v["SQ_LDS_IDX_ACTIVE"] if v["SQ_LDS_IDX_ACTIVE"] else 0,
            100 * v["SQ_WAIT_ANY"] / wc, 100 * v["SQ_WAIT_INST_ANY"] / wc,
            100 * b.get("SQ_ACTIVE_INST_ANY", 0) / wc if b else 0, rd))
    mf = sum(v["SQ_INSTS_MFMA"] for _, v in rows)
    va = sum(v["SQ_INSTS_VALU"] for _, v in rows)
    print("\nall dcg kernels: %.1f us, MFMA work %.1f GFLOP -> %.1f TFLOP/s over kernel time; "
          "non-MFMA VALU : MFMA = %.2f : 1" % (tt / 1e3, mf * FLOP / 1e9, mf * FLOP / tt / 1e3, (va - mf) / mf))


if __name__ == "__main__":
    main(sys.argv[1:])
