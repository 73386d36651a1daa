"""Decode projections at the headline's running-set size (M = 288-320 rows), weights cold (copies
cycled past the 256 MB Infinity Cache, as in a real decode step) vs hot (one copy, MALL / L2
resident): how much of a latency-bound GEMM's time is the weight fetch latency?  JSON lines."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from mxserve import ops  # noqa: E402
from mxserve.ops import decode_gemm as dg  # noqa: E402

dev = torch.device("cuda:0")
F = torch.nn.functional
shapes = {"qkv": (3072, 2048, 0), "o": (2048, 2048, 0), "gate_up": (16384, 2048, 1), "down": (2048, 8192, 0)}
for M in (288, 320):
    for name, (N, K, epi) in shapes.items():
        ws = dg.weight_copies((torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16))
        x = torch.randn(M, K, device=dev).to(torch.bfloat16)
        f = (lambda w: ops.silu_mul(F.linear(x, w))) if epi else (lambda w: F.linear(x, w))
        cold = dg._graph_time(lambda i: f(ws[i % len(ws)]))
        hot = dg._graph_time(lambda i: f(ws[0]))
        print(json.dumps({"M": M, "proj": name, "cold_us": round(cold, 2), "hot_us": round(hot, 2),
                          "hot_speedup": round(cold / hot, 3)}), flush=True)
