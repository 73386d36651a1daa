#!/usr/bin/env python3
"""Prefill projection GEMMs of Llama-3.2-1B at the headline's step sizes: hipBLASLt (torch F.linear;
addmm_ for the residual form) against gemm_pf (csrc/kernels/gemm_pf.hip) at each stream-K setting.
JSON lines: proj, M, impl, us, TFLOP/s (2 M N K / t), max error vs hipBLASLt.

  python scripts/pf_shape_probe.py [M,M,...] [proj,proj,...]
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, iters=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(5):
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3 / iters)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    from mxserve import ops
    dev = torch.device("cuda:0")
    shapes = {"qkv": (3072, 2048, 0), "o": (2048, 2048, 2), "down": (2048, 8192, 2), "gate_up": (16384, 2048, 1)}
    Ms = [int(t) for t in (sys.argv[1].split(",") if len(sys.argv) > 1 else "2048,4096,6144,6656,8192".split(","))]
    only = sys.argv[2].split(",") if len(sys.argv) > 2 else list(shapes)
    F = torch.nn.functional
    for name in only:
        N, K, epi = shapes[name]
        w = ((torch.rand(N, K, device=dev) * 2 - 1) * K ** -0.5).to(torch.bfloat16)
        for M in Ms:
            x = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
            fl = 2.0 * M * N * K
            r = torch.randn(M, N, device=dev).to(torch.bfloat16)
            if epi == 2:
                base = lambda: r.addmm_(x, w.t())  # noqa: E731
            elif epi == 1:
                base = lambda: ops.silu_mul(F.linear(x, w))  # noqa: E731
            else:
                base = lambda: F.linear(x, w)  # noqa: E731
            us = timed(base)
            print(json.dumps({"proj": name, "M": M, "N": N, "K": K, "impl": "hipblaslt", "us": round(us, 2),
                              "TF": round(fl / us / 1e6, 1)}), flush=True)
            ref = F.linear(x, w).float()
            if epi == 1:
                ref = ops.silu_mul(F.linear(x, w)).float()
            for tr in (256, 192, 160, 128):
                for mi in (0, 8, 32):
                    if epi == 2:
                        out = r.clone()
                        fn = lambda: ops.gemm_pf(x, w, 2, out, mi, resid=out, trows=tr)  # noqa: E731
                        chk = ops.gemm_pf(x, w, 2, None, mi, resid=r, trows=tr)
                        err = (chk.float() - (r.float() + ref)).abs().max().item()
                    else:
                        out = torch.empty(M, N // 2 if epi == 1 else N, device=dev, dtype=torch.bfloat16)
                        fn = lambda: ops.gemm_pf(x, w, epi, out, mi, trows=tr)  # noqa: E731
                        fn()
                        err = (out.float() - ref).abs().max().item()
                    us2 = timed(fn)
                    print(json.dumps({"proj": name, "M": M, "impl": f"gemm_pf/{tr}/{mi}", "us": round(us2, 2),
                                      "TF": round(fl / us2 / 1e6, 1), "vs_hipblaslt": round(us / us2, 3),
                                      "max_err": round(err, 4)}), flush=True)


if __name__ == "__main__":
    main()
