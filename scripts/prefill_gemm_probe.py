#!/usr/bin/env python3
"""Prefill projection GEMMs (Llama-3.2-1B shapes, T tokens): hipBLASLt through torch vs the
hand-written prefill GEMM kernel (csrc/kernels/gemm_prefill.hip, when built), timed with events over
20 back-to-back calls on random operands.  JSON lines: proj, T, impl, microseconds, TFLOP/s."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


def main():
    from mxserve import ops
    dev = torch.device("cuda:0")
    shapes = {"qkv": (3072, 2048), "o": (2048, 2048), "gate_up": (16384, 2048), "down": (2048, 8192)}
    Ts = [int(t) for t in (sys.argv[1].split(",") if len(sys.argv) > 1 else "512,1024,2048,4096,8192".split(","))]
    pg = getattr(ops, "prefill_gemm", None)
    for name, (N, K) in shapes.items():
        w = (torch.rand(N, K, device=dev) * 2 - 1).to(torch.bfloat16) * K ** -0.5
        for T in Ts:
            x = (torch.rand(T, K, device=dev) * 2 - 1).to(torch.bfloat16)
            fl = 2.0 * T * N * K
            us = timed(lambda: torch.nn.functional.linear(x, w))
            print(json.dumps({"proj": name, "T": T, "impl": "hipblaslt", "us": round(us, 2),
                              "TFLOPs": round(fl / us / 1e6, 1)}), flush=True)
            if pg is not None:
                out = torch.empty(T, N, device=dev, dtype=torch.bfloat16)
                for cfg in ops.prefill_gemm_configs(T, N, K):
                    if not pg(out, x, w, cfg):
                        continue
                    us2 = timed(lambda: pg(out, x, w, cfg))
                    err = (out.float() - torch.nn.functional.linear(x, w).float()).abs().max().item()
                    print(json.dumps({"proj": name, "T": T, "impl": "mfma", "cfg": cfg, "us": round(us2, 2),
                                      "TFLOPs": round(fl / us2 / 1e6, 1), "max_err": err}), flush=True)


if __name__ == "__main__":
    main()
