#!/usr/bin/env python3
"""Every mt-kernel configuration for a few projection shapes (graph-timed, 20 calls), hipBLASLt first:
JSON lines (proj, M, cfg, us).  Run under rocprofv3 --kernel-trace --stats to split the GEMM kernel
from its split-K reduce."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from mxserve.ops import decode_gemm as dg
    dev = torch.device("cuda:0")
    cases = [("o", 2048, 2048, 0, 64), ("qkv", 3072, 2048, 0, 256), ("gate_up", 16384, 2048, 1, 256)]
    dg.TABLE.part = torch.empty(8 * 256 * 16384, dtype=torch.float32, device=dev)
    for name, N, K, epi, M in cases:
        w = ((torch.rand(N, K, device=dev) * 2 - 1) * K ** -0.5).to(torch.bfloat16)
        x = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
        t = dg._graph_time(lambda: torch.nn.functional.linear(x, w))
        print(json.dumps({"proj": name, "M": M, "cfg": "hipblaslt", "us": round(t, 2)}), flush=True)
        out = torch.empty(M, N // 2 if epi else N, device=dev, dtype=torch.bfloat16)
        for cfg in dg.mt_candidates(M, N, K, epi, max_blocks=4096):
            if dg.TABLE.run(out, x, w, cfg, epi):
                t = dg._graph_time(lambda: dg.TABLE.run(out, x, w, cfg, epi))
                print(json.dumps({"proj": name, "M": M, "cfg": cfg, "us": round(t, 2)}), flush=True)


if __name__ == "__main__":
    main()
