"""Sampling kernel time at the headline's decode batch (448 rows x 128256 bf16 logits): greedy,
temperature 1 (the bench), top-p 0.9 + top-k 40.  JSON lines."""
import json
import os
import sys

import torch

sys.path.insert(0, os.environ.get("MXS_AB_ROOT") or os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from mxserve import ops  # noqa: E402

dev = torch.device("cuda:0")
for B in (256, 448):
    V = 128256
    logits = (torch.randn(B, V, device=dev) * 3).to(torch.bfloat16)
    seeds = torch.arange(B, device=dev)
    steps = torch.zeros(B, dtype=torch.int64, device=dev)
    for name, t, tp, tk in (("greedy", 0.0, 1.0, 0), ("t1", 1.0, 1.0, 0), ("t0.8_p0.9_k40", 0.8, 0.9, 40)):
        args = (torch.full((B,), t, device=dev), torch.full((B,), tp, device=dev),
                torch.full((B,), tk, dtype=torch.int32, device=dev), seeds, steps)
        ops.sample(logits, *args)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            ops.sample(logits, *args)
        e1.record()
        torch.cuda.synchronize()
        print(json.dumps({"B": B, "mode": name, "us": round(e0.elapsed_time(e1) * 1e3 / 20, 1)}), flush=True)
