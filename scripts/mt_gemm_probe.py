#!/usr/bin/env python3
"""Medium-M projection GEMMs (decode batches 64-256, short prefill chunks): hipBLASLt vs the glds-staged
mt kernel (csrc/kernels/gemm_decode.hip mt_gemm_kernel) vs the earlier decode kernel forms, each timed
as 20 calls replayed from one hipGraph (the decode graphs' conditions) on random operands, cycling
through copies of the weight matrix that together exceed the Infinity Cache (MXS_PROBE_COLD=0: one
cache-resident copy).  gate_up is
timed with its SiLU*mul (hipBLASLt + silu_mul kernel vs the fused epilogue).  JSON lines per
(model, proj, M): hipBLASLt us, best mt config/us, best earlier-kernel config/us, max error."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = {
    "llama-3.2-1b": {"qkv": (3072, 2048, 0), "o": (2048, 2048, 0), "gate_up": (16384, 2048, 1),
                     "down": (2048, 8192, 0)},
    "llama-3-8b": {"qkv": (6144, 4096, 0), "o": (4096, 4096, 0), "gate_up": (28672, 4096, 1),
                   "down": (4096, 14336, 0)},
    "llama-3-70b": {"qkv": (10240, 8192, 0), "o": (8192, 8192, 0), "gate_up": (57344, 8192, 1),
                    "down": (8192, 28672, 0)},
    "llama-3-70b-tp8": {"qkv": (1280, 8192, 0), "o": (8192, 1024, 0), "gate_up": (7168, 8192, 1),
                        "down": (8192, 3584, 0)},
}


COLD = os.environ.get("MXS_PROBE_COLD", "1") != "0"  # cycle weight copies past the Infinity Cache


def main():
    from mxserve.ops import decode_gemm as dg, silu_mul
    dev = torch.device("cuda:0")
    Ms = [int(m) for m in (sys.argv[1].split(",") if len(sys.argv) > 1 else "64,128,192,256,384,512".split(","))]
    models = sys.argv[2].split(",") if len(sys.argv) > 2 else list(SHAPES)
    dg.TABLE.part = torch.empty(8 * max(Ms) * 57344, dtype=torch.float32, device=dev)
    for model in models:
        for name, (N, K, epi) in SHAPES[model].items():
            w = ((torch.rand(N, K, device=dev) * 2 - 1) * K ** -0.5).to(torch.bfloat16)
            ws = dg.weight_copies(w) if COLD else [w]
            for M in Ms:
                x = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
                ref = torch.nn.functional.linear(x, w)
                ref = silu_mul(ref) if epi else ref
                lib = (lambda i: silu_mul(torch.nn.functional.linear(x, ws[i % len(ws)]))) if epi else \
                    (lambda i: torch.nn.functional.linear(x, ws[i % len(ws)]))
                t_lib = dg._graph_time(lib)
                out = torch.empty(M, N // 2 if epi else N, device=dev, dtype=torch.bfloat16)
                best = {"mt": (None, 1e9, 0.0), "old": (None, 1e9, 0.0)}
                cands = dg.mt_candidates(M, N, K, epi) + ([c for c in dg.candidates(min(M, 256), N, K, epi)
                                                           if c[0] != "mt"] if M <= 256 else [])
                for cfg in cands:
                    if not dg.TABLE.run(out, x, w, cfg, epi):
                        continue
                    err = (out.float() - ref.float()).abs().max().item()
                    t = dg._graph_time(lambda i: dg.TABLE.run(out, x, ws[i % len(ws)], cfg, epi))
                    key = "mt" if cfg[0] == "mt" else "old"
                    if t < best[key][1]:
                        best[key] = (cfg, t, err)
                wbytes = N * K * 2
                row = {"model": model, "proj": name, "M": M, "N": N, "K": K, "weights": "cold" if COLD else "cache-hot",
                       "hipblaslt_us": round(t_lib, 2),
                       "hipblaslt_TBps_w": round(wbytes / t_lib / 1e6, 2)}
                for key, (cfg, t, err) in best.items():
                    if cfg is not None:
                        row[key] = {"cfg": cfg, "us": round(t, 2), "TBps_w": round(wbytes / t / 1e6, 2),
                                    "max_err": round(err, 4), "speedup_vs_hipblaslt": round(t_lib / t, 3)}
                print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
