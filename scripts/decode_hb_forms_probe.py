#!/usr/bin/env python3
"""hipBLASLt call forms for the Llama-3.2-1B decode projections at the large decode buckets
(M = 320-448): F.linear, torch.mm into a preallocated output, rows padded to the next multiple of
64 / 128, and a two-call row split -- cold weights, hipGraph-timed like the decode-GEMM tuner.
JSON lines."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from mxserve.ops import decode_gemm as dg
    dev = torch.device("cuda:0")
    shapes = {"qkv": (3072, 2048), "o": (2048, 2048), "gate_up": (16384, 2048), "down": (2048, 8192),
              "lm_head": (128256, 2048)}
    F = torch.nn.functional
    for name, (N, K) in shapes.items():
        w = (torch.randn(N, K, device=dev) * K ** -0.5).to(torch.bfloat16)
        ws = dg.weight_copies(w)
        for M in (320, 384, 416, 448):
            x = (torch.randn(M, K, device=dev) * 0.5).to(torch.bfloat16)
            out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
            forms = {"linear": lambda i: F.linear(x, ws[i % len(ws)]),
                     "mm_out": lambda i: torch.mm(x, ws[i % len(ws)].t(), out=out)}
            for pad in (64, 128, 256):
                P = -(-M // pad) * pad
                if P != M:
                    xp = torch.zeros(P, K, dtype=torch.bfloat16, device=dev)
                    xp[:M] = x
                    forms[f"pad{P}"] = (lambda xp: lambda i: F.linear(xp, ws[i % len(ws)]))(xp)
            for a in (256, 192, 128):
                if a < M:
                    def split(i, a=a):
                        wi = ws[i % len(ws)]
                        torch.mm(x[:a], wi.t(), out=out[:a])
                        torch.mm(x[a:], wi.t(), out=out[a:])
                    forms[f"split{a}"] = split
            res = {k: round(dg._graph_time(f), 2) for k, f in forms.items()}
            best = min(res, key=res.get)
            print(json.dumps({"proj": name, "M": M, "N": N, "K": K, "us": res, "best": best,
                              "gain_vs_linear": round(res["linear"] / res[best], 3)}), flush=True)
        del ws


if __name__ == "__main__":
    main()
