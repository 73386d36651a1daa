#!/usr/bin/env python3
"""Pretty-print scripts/pf_shape_probe.py JSON lines: one row per (proj, M) with hipBLASLt and every
gemm_pf setting in TFLOP/s (x vs hipBLASLt)."""
import json
import sys

for path in sys.argv[1:]:
    print(f"== {path}")
    for ln in open(path):
        if not ln.startswith("{"):
            continue
        r = json.loads(ln)
        if r["impl"] == "hipblaslt":
            print(f"\n{r['proj']:8s} M={r['M']:5d} hipblaslt {r['us']:8.2f} us {r['TF']:7.1f} TF", end="")
        else:
            print(f" | {r['impl'][8:]}: {r['TF']:6.1f} ({r['vs_hipblaslt']:.2f}x)", end="")
    print()
