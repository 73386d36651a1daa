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
    ap.add_argument("--by-grid", default="", help="also break kernels whose name contains this down by grid size")
    ap.add_argument("--busy", type=float, default=0.0,
                    help="print the GPU-busy fraction (union of kernel intervals) per bin of this many seconds")
    ap.add_argument("--exclusive", action="store_true",
                    help="per kernel family, time with concurrent kernels' overlap split evenly among them "
                         "(kernels on side streams overlap; raw durations then over-count)")
    a = ap.parse_args()
    db = sqlite3.connect(a.db)
    if a.exclusive:
        exclusive(db)
        return
    if a.busy:
        iv = db.execute("select start, end from kernels order by start").fetchall()
        t0, t1 = iv[0][0], max(e for _, e in iv)
        binw = int(a.busy * 1e9)
        nb = (t1 - t0) // binw + 1
        busy = [0] * nb
        cs, ce = iv[0]
        def add(s_, e_):
            while s_ < e_:
                b = (s_ - t0) // binw
                be = t0 + (b + 1) * binw
                busy[b] += min(e_, be) - s_
                s_ = min(e_, be)
        for s_, e_ in iv[1:]:
            if s_ > ce:
                add(cs, ce)
                cs, ce = s_, e_
            else:
                ce = max(ce, e_)
        add(cs, ce)
        print("-- GPU busy per bin (union of kernel intervals)")
        for i, b in enumerate(busy):
            print(f"{i * a.busy:7.1f}s  {100.0 * b / binw:6.2f}%")
    cols = [r[1] for r in db.execute("pragma table_info(kernels)").fetchall()]
    if a.by_grid:
        gx = next((c for c in cols if c.lower() in ("grid_size_x", "grid_x", "grid_size")), None)
        gy = next((c for c in cols if c.lower() in ("grid_size_y", "grid_y")), None)
        wx = next((c for c in cols if c.lower() in ("workgroup_size_x", "workgroup_x", "workgroup_size")), None)
        if gx is None:
            print("columns:", cols)
        else:
            q = (f"select name, {gx}, {gy or 0}, {wx or 0}, count(*), sum(end - start) from kernels where name like ? "
                 f"group by name, {gx}, {gy or 0} order by 6 desc")
            tot = db.execute("select sum(end - start) from kernels").fetchone()[0]
            print(f"-- by grid ({a.by_grid})")
            for n, x, y, w, c, t in db.execute(q, (f"%{a.by_grid}%",)).fetchall()[:a.top]:
                print(f"{100.0 * t / tot:6.2f}%  {c:7d} calls  {t / 1e3 / c:9.2f} us  grid {x}x{y} wg {w}  {n[:90]}")
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


def family(name: str) -> str:
    if name.startswith(("Cijk", "Custom_Cijk")):
        return "hipblaslt"
    n = name.split("(")[0].replace("void ", "")
    return n.split("<")[0]


def exclusive(db) -> None:
    """Sweep the kernel intervals: each slice between consecutive start / end events is shared evenly
    by the kernels active in it; a family's exclusive time is the sum of its shares, and the shares add
    up to the GPU-busy time (the union of the intervals)."""
    iv = db.execute("select name, start, end from kernels").fetchall()
    ev = []
    for i, (n, s_, e_) in enumerate(iv):
        ev.append((s_, 1, i))
        ev.append((e_, 0, i))
    ev.sort()
    active, t_prev, share, raw = set(), None, {}, {}
    for n, s_, e_ in iv:
        f = family(n)
        raw[f] = raw.get(f, 0) + (e_ - s_)
    for t, kind, i in ev:
        if active and t_prev is not None and t > t_prev:
            d = (t - t_prev) / len(active)
            for j in active:
                f = family(iv[j][0])
                share[f] = share.get(f, 0.0) + d
        t_prev = t
        if kind:
            active.add(i)
        else:
            active.discard(i)
    busy, tot_raw = sum(share.values()), sum(raw.values())
    print(f"# busy {busy / 1e6:.1f} ms (union of kernel intervals), raw kernel time {tot_raw / 1e6:.1f} ms "
          f"(overlap {100.0 * (tot_raw - busy) / busy:.1f} %)")
    print("# family: exclusive share of busy time | raw-duration share")
    for f, v in sorted(share.items(), key=lambda kv: -kv[1]):
        print(f"{100.0 * v / busy:6.2f}%  {100.0 * raw[f] / tot_raw:6.2f}%  {f}")


if __name__ == "__main__":
    main()
