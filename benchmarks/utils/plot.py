"""Plots for benchmark output: throughput vs TTFT / ITL per concurrency and request-rate point.

    python3 -m benchmarks.utils.plot --data-dir DIR     (DIR/<name>/summary.json, any number of names)
Writes DIR/plots/*.png (matplotlib, Agg backend) and a markdown table DIR/plots/summary.md.
"""
from __future__ import annotations

import argparse
import glob
import json
import os


def load(data_dir: str) -> dict:
    out = {}
    for p in sorted(glob.glob(os.path.join(data_dir, "*", "summary.json"))):
        with open(p) as f:
            d = json.load(f)
        out[d["benchmark"]] = d["points"]
    return out


def main(argv=None) -> None:
    ap = argparse.ArgumentParser(prog="python3 -m benchmarks.utils.plot")
    ap.add_argument("--data-dir", required=True)
    a = ap.parse_args(argv)
    runs = load(a.data_dir)
    pdir = os.path.join(a.data_dir, "plots")
    os.makedirs(pdir, exist_ok=True)
    rows = ["| benchmark | mode | x | output tok/s | req/s | TTFT p50 ms | ITL p50 ms | failed |", "|---" * 8 + "|"]
    for name, pts in runs.items():
        for p in pts:
            x = p.get("concurrency", p.get("request_rate"))
            rows.append(f"| {name} | {p['mode']} | {x} | {p['output_tok_per_s']:.1f} | {p['requests_per_s']:.2f} | "
                        f"{p['ttft_ms_p50'] or float('nan'):.1f} | {p['itl_ms_p50'] or float('nan'):.2f} | {p['failed']} |")
    with open(os.path.join(pdir, "summary.md"), "w") as f:
        f.write("\n".join(rows) + "\n")
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    for metric, label in (("ttft_ms_p50", "TTFT p50 (ms)"), ("itl_ms_p50", "ITL p50 (ms)")):
        fig, ax = plt.subplots(figsize=(7, 4.5))
        for name, pts in runs.items():
            pts = [p for p in pts if p.get(metric) is not None]
            ax.plot([p[metric] for p in pts], [p["output_tok_per_s"] for p in pts], marker="o", label=name)
        ax.set_xlabel(label)
        ax.set_ylabel("output tok/s")
        ax.grid(alpha=0.3)
        ax.legend()
        fig.tight_layout()
        fig.savefig(os.path.join(pdir, f"throughput_vs_{metric}.png"), dpi=120)
        plt.close(fig)
    print(f"plots written to {pdir}")


if __name__ == "__main__":
    main()
