#!/usr/bin/env python3
"""ops.linear with the persisted M plans vs one F.linear at mixed-step row counts (Llama-3.2-1B
projections), interleaved rounds; JSON lines with both times and the plan used."""
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
    from mxserve import ops
    dev = torch.device("cuda:0")
    shapes = {"qkv": (3072, 2048), "o": (2048, 2048), "gate_up": (16384, 2048), "down": (2048, 8192)}
    for M in (4270, 4350, 4480, 3300, 6144, 6700, 8192, 2600):
        for name, (N, K) in shapes.items():
            x = torch.randn(M, K, device=dev).to(torch.bfloat16)
            w = (torch.randn(N, K, device=dev) * K ** -0.5).to(torch.bfloat16)
            ref = torch.nn.functional.linear(x, w)
            got = ops.linear(x, w)
            err = float((got.float() - ref.float()).abs().max())
            a, b = [], []
            for _ in range(3):
                a.append(timed(lambda: torch.nn.functional.linear(x, w)))
                b.append(timed(lambda: ops.linear(x, w)))
            print(json.dumps({"proj": name, "M": M, "plan": ops._mplan(M, N, K, dev), "linear_us": round(min(a), 2),
                              "ops_linear_us": round(min(b), 2), "max_abs_err": err}), flush=True)


if __name__ == "__main__":
    main()
