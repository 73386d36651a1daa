#!/usr/bin/env python3
"""GPU busy fraction from a rocprofv3 rocpd database: the union of kernel intervals over a window
(default: the last `--window` seconds of kernel activity), i.e. how much of the wall the device
executed anything, plus the largest idle gaps.  `python scripts/gpu_busy.py DB [--window 8]`

--attribute: also group the idle time in gaps over 50 us by the kernels on either side of the gap
(short names), and split the busy time by kernel family, so a gap can be traced to the step phase
that leaves the device waiting (late admission, an eager prefill launch, a host sync)."""
import argparse
import json
import re
import sqlite3
from collections import defaultdict


def short(name: str) -> str:
    n = re.sub(r"\(.*", "", name or "?")
    n = re.sub(r"<.*", "", n)
    n = n.split("::")[-1]
    if n.startswith("Cijk_") or n.startswith("Custom_Cijk"):
        m = re.search(r"MT(\d+x\d+x\d+)", name)
        return "hipblaslt_" + (m.group(1) if m else "?")
    return n[:48]


def family(name: str) -> str:
    s = short(name)
    for key, fam in (("paged_decode", "decode_attention"), ("paged_prefill", "prefill_attention"),
                     ("hipblaslt", "hipblaslt"), ("mt_gemm", "hand_gemm"), ("decode_gemm", "hand_gemm"),
                     ("prefill_gemm", "hand_gemm"), ("gemm_big", "hand_gemm"), ("splitk", "epilogue"),
                     ("rope", "rope_cache"), ("rmsnorm", "norm"), ("rms_norm", "norm"), ("silu", "silu_mul"),
                     ("sample", "sampling"), ("allreduce", "collective"), ("moe", "moe")):
        if key in s:
            return fam
    return "other:" + s[:32]


def kernel_rows(db):
    cols = [r[1] for r in db.execute("pragma table_info(kernels)").fetchall()]
    name_col = next((c for c in ("name", "kernel_name", "KernelName") if c in cols), None)
    q = f"select start, end, {name_col} from kernels" if name_col else "select start, end, '' from kernels"
    return sorted(db.execute(q).fetchall())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--window", type=float, default=8.0)
    ap.add_argument("--attribute", action="store_true")
    a = ap.parse_args()
    db = sqlite3.connect(a.db)
    rows = kernel_rows(db)
    t_end = max(e for _, e, _ in rows)
    t_lo = t_end - a.window * 1e9
    rows = [(max(s, t_lo), e, n) for s, e, n in rows if e > t_lo]
    busy, cur_s, cur_e, gaps = 0, None, None, []
    prev_name = None
    gap_by_pair: dict = defaultdict(lambda: [0, 0.0])
    fam_busy: dict = defaultdict(float)
    for s, e, n in rows:
        fam_busy[family(n)] += e - s
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
                g = s - cur_e
                gaps.append(g)
                if g > 50e3:
                    k = f"{short(prev_name)} -> {short(n)}"
                    gap_by_pair[k][0] += 1
                    gap_by_pair[k][1] += g / 1e6
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
        prev_name = n
    busy += cur_e - cur_s
    span = t_end - rows[0][0]
    gaps.sort(reverse=True)
    out = {"window_s": round(span / 1e9, 3), "busy_fraction": round(busy / span, 4),
           "kernels": len(rows), "idle_ms": round((span - busy) / 1e6, 2),
           "gaps_over_50us": sum(1 for g in gaps if g > 50e3),
           "idle_ms_in_gaps_over_50us": round(sum(g for g in gaps if g > 50e3) / 1e6, 2),
           "largest_gaps_us": [round(g / 1e3, 1) for g in gaps[:10]]}
    if a.attribute:
        tot = sum(fam_busy.values())
        out["kernel_time_share"] = {k: round(v / tot, 4) for k, v in sorted(fam_busy.items(), key=lambda kv: -kv[1])[:16]}
        out["gap_ms_by_neighbours"] = {k: [c, round(ms, 2)] for k, (c, ms) in
                                       sorted(gap_by_pair.items(), key=lambda kv: -kv[1][1])[:12]}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
