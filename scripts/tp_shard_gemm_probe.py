#!/usr/bin/env python3
"""Every decode-GEMM candidate (mxserve/ops/decode_gemm.py) vs hipBLASLt on Llama-3-70B TP-8 shard
shapes at small batches, cold weights, hipGraph-timed (the tuner's own clock); the top candidates per
case with their effective weight-streaming rate.  JSON lines."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from mxserve.ops import decode_gemm as dg
    dev = torch.device("cuda:0")
    shapes = {"qkv_tp8": (1280, 8192, 0), "o_tp8": (8192, 1024, 0), "down_tp8": (8192, 3584, 0),
              "gate_up_tp8": (7168, 8192, 1)}
    only = [a for a in sys.argv[1:] if a in shapes]
    for name, (N, K, epi) in shapes.items():
        if only and name not in only:
            continue
        w = (torch.randn(N, K, device=dev) * K ** -0.5).to(torch.bfloat16)
        ws = dg.weight_copies(w)
        dg.TABLE.part = torch.empty(32 * 64 * N, dtype=torch.float32, device=dev)
        for M in (1, 8, 32, 64):
            x = (torch.randn(M, K, device=dev) * 0.5).to(torch.bfloat16)
            out = torch.empty(M, N // 2 if epi else N, dtype=torch.bfloat16, device=dev)
            if epi:  # hipBLASLt + the SiLU*mul kernel, as the engine runs it
                from mxserve.ops import silu_mul
                t_lib = dg._graph_time(lambda i: silu_mul(torch.nn.functional.linear(x, ws[i % len(ws)])))
            else:
                t_lib = dg._graph_time(lambda i: torch.nn.functional.linear(x, ws[i % len(ws)]))
            res = []
            for cfg in dg.candidates(M, N, K, epi):
                if not dg.TABLE.run(out, x, w, cfg, epi):
                    continue
                t = dg._graph_time(lambda i, c=cfg: dg.TABLE.run(out, x, ws[i % len(ws)], c, epi))
                tn = dg._graph_time(lambda i, c=cfg: dg.TABLE.run(out, x, ws[i % len(ws)], c, 0, reduce=False)) \
                    if dg.TABLE.splitk(cfg) > 1 and not epi else t
                res.append((t, tn, cfg))
            res.sort(key=lambda r: r[0])
            by = N * K * 2
            print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "epi": epi, "hipblaslt_us": round(t_lib, 2),
                              "hipblaslt_TBps": round(by / t_lib / 1e6, 2), "n_cands": len(res),
                              "top": [{"cfg": list(c), "us": round(t, 2), "TBps": round(by / t / 1e6, 2),
                                       "no_reduce_us": round(tn, 2)} for t, tn, c in res[:5]]}), flush=True)
        del ws


if __name__ == "__main__":
    main()
