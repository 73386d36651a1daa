#!/usr/bin/env python3
"""gemm_w4 (four waves, 128 x 128 per wave) against gemm_pf (eight waves, stream-K; its best
(rows, min_iters) here) and hipBLASLt on the Llama-3.2-1B prefill projections at headline row
counts.  Interleaved rounds in one process, medians (cdna_hip_programming.md §5.4 rule 24); random
[-1, 1) operands (rule 25).  One JSON line per (projection, M)."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from mxserve import ops  # noqa: E402

SHAPES = [("qkv", 3072, 2048, 0), ("o", 2048, 2048, 2), ("gate_up", 16384, 2048, 1), ("down", 2048, 8192, 2)]
PF_CFGS = [(256, 0), (256, 8), (256, 16), (224, 0), (224, 16), (192, 0), (192, 32), (160, 0), (128, 0)]


def timed(fn, iters=10):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


def main():
    dev = torch.device("cuda:0")
    Ms = [int(m) for m in os.environ.get("W4_MS", "2048,4096,6592,8192").split(",")]
    rounds = int(os.environ.get("W4_ROUNDS", "5"))
    only = [s for s in os.environ.get("W4_PROJ", "").split(",") if s]
    for name, N, K, epi in SHAPES:
        if only and name not in only:
            continue
        w = ((torch.rand(N, K, device=dev) * 2 - 1) * K ** -0.5).to(torch.bfloat16)
        for M in Ms:
            x = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
            r = (torch.rand(M, N, device=dev) * 2 - 1).to(torch.bfloat16) if epi == 2 else None
            out = torch.empty(M, N // 2 if epi == 1 else N, device=dev, dtype=torch.bfloat16)
            cands = {"w4": lambda: ops.gemm_w4(x, w, epi, out, resid=r)}
            for tr, mi in PF_CFGS:
                cands[f"pf{tr}/{mi}"] = (lambda tr=tr, mi=mi: ops.gemm_pf(x, w, epi, out, mi, resid=r, trows=tr))
            if epi == 0:
                cands["hipblaslt"] = lambda: torch.nn.functional.linear(x, w)
            elif epi == 1:
                cands["hipblaslt"] = lambda: ops.silu_mul(torch.nn.functional.linear(x, w))
            else:
                rr = r.clone()
                cands["hipblaslt"] = lambda: rr.addmm_(x, w.t())
            # correctness of w4 against the fp32 product
            ref = x.float() @ w.float().t()
            if epi == 1:
                ref = torch.nn.functional.silu(ref[:, :N // 2]) * ref[:, N // 2:]
            elif epi == 2:
                ref = ref + r.float()
            assert ops.gemm_w4(x, w, epi, out, resid=r) is not None
            err = ((out.float() - ref).abs().max() / ref.abs().max().clamp(min=1)).item()
            ts = {k: [] for k in cands}
            for _ in range(rounds):
                for k, fn in cands.items():
                    ts[k].append(timed(fn))
            med = {k: round(statistics.median(v), 2) for k, v in ts.items()}
            best_pf = min((k for k in med if k.startswith("pf")), key=med.get)
            fl = 2.0 * M * N * K
            print(json.dumps({"proj": name, "M": M, "N": N, "K": K, "epi": epi, "w4_rel_err": round(err, 5),
                              "us": med, "w4_TF": round(fl / med["w4"] / 1e6, 1),
                              "pf_best": best_pf, "pf_TF": round(fl / med[best_pf] / 1e6, 1),
                              "hipblaslt_TF": round(fl / med["hipblaslt"] / 1e6, 1),
                              "w4_vs_hipblaslt": round(med["hipblaslt"] / med["w4"], 3),
                              "w4_vs_pf": round(med[best_pf] / med["w4"], 3)}), flush=True)


if __name__ == "__main__":
    main()
