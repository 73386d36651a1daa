#!/usr/bin/env python3
"""Every decode-GEMM kernel configuration vs hipBLASLt at the Llama-3.2-1B projection shapes, timed
inside hipGraphs (20 calls per replay).  JSON lines: shape, M, config, microseconds, weight GB/s.
  python scripts/decode_gemm_probe.py [M,M,...] [proj,proj,...]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from mxserve.ops import decode_gemm as dg
    from mxserve import ops
    dev = torch.device("cuda:0")
    shapes = {"qkv": (3072, 2048, 0), "o": (2048, 2048, 0), "gate_up": (16384, 2048, 1), "down": (2048, 8192, 0),
              "lm_head": (128256, 2048, 0)}
    Ms = [int(m) for m in (sys.argv[1].split(",") if len(sys.argv) > 1 else "256,192,128,64,16,1".split(","))]
    dg.TABLE.part = torch.empty(8 * 256 * 128256, dtype=torch.float32, device=dev)
    only = sys.argv[2].split(",") if len(sys.argv) > 2 else list(shapes)
    for name, (N, K, epi) in shapes.items():
        if name not in only:
            continue
        w = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
        for M in Ms:
            x = torch.randn(M, K, device=dev).to(torch.bfloat16)
            f = (lambda: ops.silu_mul(torch.nn.functional.linear(x, w))) if epi else (
                lambda: torch.nn.functional.linear(x, w))
            t = dg._graph_time(f)
            res = [("hipblaslt", t)]
            out = torch.empty(M, N // 2 if epi else N, device=dev, dtype=torch.bfloat16)
            for cfg in dg.candidates(M, N, K, epi, all_mf=True):
                res.append((cfg, dg._graph_time(lambda: dg.TABLE.run(out, x, w, cfg, epi))))
            res.sort(key=lambda r: r[1])
            for c, us in res[:6]:
                print(json.dumps({"proj": name, "M": M, "cfg": c, "us": round(us, 2),
                                  "GBps_w": round(N * K * 2 / us / 1e3, 1)}), flush=True)


if __name__ == "__main__":
    main()
