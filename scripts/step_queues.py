"""Print the last full training step of a rocprofv3 kernel trace with each dispatch's hardware
queue: start (us from the step's first kernel), duration, queue, grid and kernel name.

    python scripts/step_queues.py gpurun_out/prof_<tag>/run_results.db [--marker adam2]
"""
import argparse
import re
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--marker", default="adam2", help="kernel that ends a step")
    a = ap.parse_args()
    cur = sqlite3.connect(a.db).cursor()
    rows = [r for r in cur.execute("select name, start, end, queue_id, grid_x, grid_y from kernels order by start")
            if "dcg" in r[0]]
    ends = [i for i, r in enumerate(rows) if a.marker in r[0]]
    lo, hi = ends[-2] + 1, ends[-1] + 1
    t0 = rows[lo][1]
    for n, s, e, q, gx, gy in rows[lo:hi]:
        nm = re.sub(r"^_ZN3dcg\d+", "", n)[:60]
        print("%8.1f %6.1f q%-3s g(%d,%d) %s" % ((s - t0) / 1000, (e - s) / 1000, q, gx, gy, nm))
    print("span %.1f us" % ((rows[hi - 1][2] - t0) / 1000))


if __name__ == "__main__":
    main()
