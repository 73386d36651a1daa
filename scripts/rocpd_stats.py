#!/usr/bin/env python3
"""Per-kernel statistics from a rocprofv3 rocpd database (ROCm 7.2 writes `<dir>/<name>_results.db`
by default): name, calls, total / mean us, share.  `python scripts/rocpd_stats.py DB [--per N] [--csv OUT]`
--per N divides totals by N (e.g. per iteration of a profiled loop)."""
import argparse
import csv
import sqlite3
import sys


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--per", type=float, default=1.0)
    ap.add_argument("--csv", default="")
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    db = sqlite3.connect(a.db)
    rows = db.execute("select name, count(*), sum(end - start) from kernels group by name order by 3 desc").fetchall()
    tot = sum(r[2] for r in rows)
    out = [(n, c, t / 1e3, t / 1e3 / c, 100.0 * t / tot) for n, c, t in rows]
    w = csv.writer(open(a.csv, "w") if a.csv else sys.stdout)
    if a.csv:
        w.writerow(["Name", "Calls", "TotalUs", "MeanUs", "Percentage"])
        for r in out:
            w.writerow([r[0], r[1], round(r[2], 2), round(r[3], 3), round(r[4], 2)])
    print(f"total {tot / 1e3 / a.per:.1f} us per unit ({a.per:g} units)")
    for n, c, t, m, p in out[:a.top]:
        print(f"{p:6.2f}%  {t / a.per:9.1f} us/unit  {c / a.per:7.1f} calls/unit  {m:8.2f} us  {n[:110]}")


if __name__ == "__main__":
    main()
