"""gemm_pf (persistent 256-wide tiles, stream-K) at decode batch sizes against hipBLASLt and the
table's mt choice, Llama-3.2-1B projections, cold weights (copies cycled past the Infinity Cache),
hipGraph-timed.  JSON lines.   python scripts/probes/pf_decode_probe.py [M,M..] [proj,..]"""
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
Ms = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "256,320,384,448").split(",")]
only = sys.argv[2].split(",") if len(sys.argv) > 2 else list(shapes)
dg.TABLE.part = torch.empty(16 * 448 * 16384, dtype=torch.float32, device=dev)
for name in only:
    N, K, epi = shapes[name]
    ws = dg.weight_copies((torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16))
    for M in Ms:
        x = torch.randn(M, K, device=dev).to(torch.bfloat16)
        out = torch.empty(M, N // 2 if epi else N, device=dev, dtype=torch.bfloat16)
        if epi:
            base = lambda i: ops.silu_mul(F.linear(x, ws[i % len(ws)]))  # noqa: E731
        else:
            base = lambda i: F.linear(x, ws[i % len(ws)])  # noqa: E731
        res = [("hipblaslt", dg._graph_time(base))]
        for cfg in dg.mt_candidates(M, N, K, epi)[:0] + [c for c in dg.candidates(M, N, K, epi) if c[0] == "mt"]:
            pass
        mts = [c for c in dg.candidates(M, N, K, epi) if c[0] == "mt"]
        best_mt = None
        for cfg in mts:
            t = dg._graph_time(lambda i: dg.TABLE.run(out, x, ws[i % len(ws)], cfg, epi))
            if best_mt is None or t < best_mt[1]:
                best_mt = (cfg, t)
        if best_mt:
            res.append(best_mt)
        for tr in (256, 192, 160, 128):
            for mi in (0, 2, 4, 8, 16):
                t = dg._graph_time(lambda i: ops.gemm_pf(x, ws[i % len(ws)], epi, out, mi, trows=tr))
                res.append((f"pf/{tr}/{mi}", t))
        ref = (ops.silu_mul(F.linear(x, ws[0])) if epi else F.linear(x, ws[0])).float()
        chk = torch.empty_like(out)
        best = min(res, key=lambda r: r[1])
        if str(best[0]).startswith("pf/"):
            _, tr, mi = best[0].split("/")
            ops.gemm_pf(x, ws[0], epi, chk, int(mi), trows=int(tr))
            err = (chk.float() - ref).abs().max().item()
        else:
            err = None
        res.sort(key=lambda r: r[1])
        print(json.dumps({"proj": name, "M": M, "hipblaslt_us": round(res[[r[0] for r in res].index("hipblaslt")][1], 2),
                          "best": [(str(c), round(t, 2)) for c, t in res[:5]], "best_err": err}), flush=True)
