#!/usr/bin/env python3
"""Decode-bucket GEMMs: F.linear vs torch.mm(out=) (hipBLASLt may pick different kernels for the two
call forms), each 20 calls replayed from one hipGraph on cold weight copies, as the decode tuner
times them (ops/decode_gemm.py).  JSON lines."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from mxserve.ops.decode_gemm import _graph_time, weight_copies
    dev = torch.device("cuda:0")
    shapes = {"qkv": (3072, 2048), "o": (2048, 2048), "gate_up": (16384, 2048), "down": (2048, 8192),
              "lm_head": (128256, 2048)}
    for name, (N, K) in shapes.items():
        w = (torch.randn(N, K, device=dev) * K ** -0.5).to(torch.bfloat16)
        ws = weight_copies(w)
        for M in (32, 64, 128, 192, 256, 320, 384):
            x = torch.randn(M, K, device=dev).to(torch.bfloat16)
            y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            lin = min(_graph_time(lambda i: torch.nn.functional.linear(x, ws[i % len(ws)])) for _ in range(3))
            mm = min(_graph_time(lambda i: torch.mm(x, ws[i % len(ws)].t(), out=y)) for _ in range(3))
            print(json.dumps({"proj": name, "M": M, "linear_us": round(lin, 2), "mm_out_us": round(mm, 2),
                              "mm_gain": round(1 - mm / lin, 3)}), flush=True)
        del ws


if __name__ == "__main__":
    main()
