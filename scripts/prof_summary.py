#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace SQLite database (rocpd schema).

usage: prof_summary.py <results.db> [--per-step N_KERNELS_PER_STEP] [--last-steps K]

Prints (1) totals per kernel name, (2) the dispatch sequence of the last step with grid
sizes and durations, so each op of the recorded training program can be attributed.
"""
import argparse
import collections
import re
import sqlite3


def short(name: str) -> str:
    name = re.sub(r"\(.*\)$", "", name)
    name = name.replace("void ", "")
    return name[:90]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--steps", type=int, default=0, help="timed steps at the end of the trace")
    ap.add_argument("--match", default="dcg", help="substring of our kernels (mangled names too)")
    ap.add_argument("--marker", default="linear_fwd_kernel", help="first kernel of a training step")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, duration, grid_x, grid_y, grid_z, workgroup_x, vgpr_count, accum_vgpr_count, "
                     "lds_size, start from kernels order by start").fetchall()
    ours = [r for r in rows if a.match in r[0]]
    print("total dispatches %d, ours %d" % (len(rows), len(ours)))
    tot = collections.defaultdict(lambda: [0, 0.0])
    for r in ours:
        k = short(r[0])
        tot[k][0] += 1
        tot[k][1] += r[1] / 1e3
    grand = sum(v[1] for v in tot.values())
    print("\n%-90s %6s %10s %6s" % ("kernel", "count", "total_us", "share"))
    for k, (n, t) in sorted(tot.items(), key=lambda kv: -kv[1][1]):
        print("%-90s %6d %10.1f %5.1f%%" % (k, n, t, 100 * t / grand))
    if a.steps:
        per = len(ours) // max(1, a.steps + 0)
        # find the period: number of dispatches of the first kernel in the step (philox)
        # first kernel of every training step: the G projection (it also generates z); older
        # traces started the step with the standalone Philox kernel
        first = [i for i, r in enumerate(ours) if a.marker in r[0]]
        if len(first) < 2:
            first = [i for i, r in enumerate(ours) if "philox" in r[0]]
        if len(first) >= 2:
            per = first[-1] - first[-2]
            last = ours[first[-2]:first[-1]]
            span = (last[-1][9] + last[-1][1] - last[0][9]) / 1e3
            busy = sum(r[1] for r in last) / 1e3
            print("\nlast full step: %d kernels, busy %.1f us, span %.1f us" % (len(last), busy, span))
            t0 = last[0][9]
            print("  start_us   dur_us  grid / resources / kernel")
            for r in last:
                print("%9.1f %8.1f  grid(%d,%d,%d) vgpr %d lds %d  %s" % ((r[9] - t0) / 1e3, r[1] / 1e3,
                                                                       r[2] // max(1, r[5]), r[3], r[4], r[6], r[8],
                                                                       short(r[0])))


if __name__ == "__main__":
    main()
