#!/usr/bin/env python3
"""GPU busy fraction from a rocprofv3 rocpd database: the union of kernel intervals over a window
(default: the last `--window` seconds of kernel activity), i.e. how much of the wall the device
executed anything, plus the largest idle gaps.  `python scripts/gpu_busy.py DB [--window 8]`"""
import argparse
import json
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--window", type=float, default=8.0)
    a = ap.parse_args()
    db = sqlite3.connect(a.db)
    iv = sorted(db.execute("select start, end from kernels").fetchall())
    t_end = max(e for _, e in iv)
    t_lo = t_end - a.window * 1e9
    iv = [(max(s, t_lo), e) for s, e in iv if e > t_lo]
    busy, cur_s, cur_e, gaps = 0, None, None, []
    for s, e in iv:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
                gaps.append(s - cur_e)
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    span = t_end - iv[0][0]
    gaps.sort(reverse=True)
    print(json.dumps({"window_s": round(span / 1e9, 3), "busy_fraction": round(busy / span, 4),
                      "kernels": len(iv), "idle_ms": round((span - busy) / 1e6, 2),
                      "gaps_over_50us": sum(1 for g in gaps if g > 50e3),
                      "idle_ms_in_gaps_over_50us": round(sum(g for g in gaps if g > 50e3) / 1e6, 2),
                      "largest_gaps_us": [round(g / 1e3, 1) for g in gaps[:10]]}))


if __name__ == "__main__":
    main()
