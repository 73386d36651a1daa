#!/usr/bin/env python3
"""hipBLASLt (torch F.linear) time across prefill row counts for the Llama-3.2-1B projections: is the
rate smooth in M, or do some row counts pick a poor kernel (then padding M to a multiple of 256
pays)?  JSON lines: proj, M, us, TF, and the time at M rounded up to a multiple of 256."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    dev = torch.device("cuda:0")
    shapes = {"qkv": (3072, 2048), "o": (2048, 2048), "gate_up": (16384, 2048), "down": (2048, 8192)}
    if os.environ.get("SWEEP_SHAPES") == "lm_head":  # the LM head of a decode / mixed step (M = sampled rows)
        shapes = {"lm_head": (128256, 2048)}
    Ms = [int(a) for a in sys.argv[1:]] or list(range(128, 8705, 128)) + [4300, 4270, 4200, 3300, 3170]
    ws = {k: (torch.randn(n, kk, device=dev) * kk ** -0.5).to(torch.bfloat16) for k, (n, kk) in shapes.items()}
    xmax = {k: torch.randn(max(8960, max(Ms) + 256), kk, device=dev).to(torch.bfloat16) for k, (n, kk) in shapes.items()}
    out = []
    for M in sorted(set(Ms)):
        Mp = -(-M // 256) * 256
        for name, (N, K) in shapes.items():
            x, xp = xmax[name][:M], xmax[name][:Mp]
            t = timed(lambda: torch.nn.functional.linear(x, ws[name]))
            tp = timed(lambda: torch.nn.functional.linear(xp, ws[name])) if Mp != M else t
            y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            tmm = timed(lambda: torch.mm(x, ws[name].t(), out=y))  # the split path's call form
            r = {"proj": name, "N": N, "K": K, "M": M, "us": round(t, 2), "TF": round(2 * M * N * K / t / 1e6, 1),
                 "M_pad256": Mp, "us_pad": round(tp, 2), "us_mm_out": round(tmm, 2)}
            out.append(r)
            print(json.dumps(r), flush=True)
    os.makedirs("gpurun_out", exist_ok=True)
    with open(os.environ.get("SWEEP_OUT", "gpurun_out/hipblaslt_m_sweep.jsonl"), "w") as f:
        for r in out:
            f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
