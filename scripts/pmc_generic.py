#!/usr/bin/env python3
"""Per-kernel sums of any rocprofv3 counter pass: usage pmc_generic.py <counter_collection.csv>
[--top N]. Prints dispatch count, time and every counter per kernel; with TCC_HIT_sum /
TCC_MISS_sum also the L2 hit rate."""
import csv
import sys
from collections import defaultdict


def main(argv):
    top = 30
    if "--top" in argv:
        i = argv.index("--top"); top = int(argv[i + 1]); argv = argv[:i] + argv[i + 2:]
    disp = {}
    for row in csv.DictReader(open(argv[0])):
        d = disp.setdefault(row["Dispatch_Id"], {"name": row["Kernel_Name"],
                                                 "t": int(row["End_Timestamp"]) - int(row["Start_Timestamp"])})
        d[row["Counter_Name"]] = d.get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
    agg = defaultdict(lambda: defaultdict(float))
    for d in disp.values():
        if "dcg" not in d["name"]:
            continue
        k = agg[d["name"].replace("void ", "").split("(")[0][:60]]
        k["n"] += 1
        for c, v in d.items():
            if c != "name":
                k[c] += v
    names = sorted({c for v in agg.values() for c in v} - {"n", "t"})
    print("%-60s %4s %8s %s%s" % ("kernel", "n", "us", " ".join("%14s" % c[:14] for c in names),
                                 "  L2hit" if "TCC_HIT_sum" in names else ""))
    for name, v in sorted(agg.items(), key=lambda kv: -kv[1]["t"])[:top]:
        hit = ""
        if "TCC_HIT_sum" in names:
            h, m = v["TCC_HIT_sum"], v["TCC_MISS_sum"]
            hit = "  %5.1f%%" % (100 * h / (h + m)) if h + m else "      -"
        print("%-60s %4d %8.1f %s%s" % (name, v["n"], v["t"] / 1e3, " ".join("%14.4g" % (v[c] / v["n"]) for c in names), hit))


if __name__ == "__main__":
    main(sys.argv[1:])
