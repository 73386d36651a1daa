#!/usr/bin/env python3
"""hipBLASLt solution sweep on the Llama-3.2-1B prefill projections (csrc/kernels/hblt.cpp): every
solution that supports the shape, screened with one short timing each, the best 8 re-timed in
interleaved rounds against the torch call the engine makes today (F.linear, or addmm_ into the
residual for o / down) and gemm_pf's best height.  Medians (cdna_hip_programming.md §5.4 rule 24),
random [-1, 1) operands (rule 25).  One JSON line per (projection, M)."""
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from mxserve import ops  # noqa: E402

SHAPES = [("qkv", 3072, 2048, False), ("o", 2048, 2048, True), ("down", 2048, 8192, True),
          ("gate_up", 16384, 2048, False)]


GRAPH = os.environ.get("HB_GRAPH", "0") == "1"  # time hipGraph replays (decode sizes: no host overhead)


def timed(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if GRAPH:
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s):
                for _ in range(iters):
                    fn()
        torch.cuda.current_stream().wait_stream(s)
        g.replay()
        e0.record()
        for _ in range(3):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / (3 * iters)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


def main():
    dev = torch.device("cuda:0")
    Ms = [int(m) for m in os.environ.get("HB_MS", "2048,4096,6144,6592").split(",")]
    only = [s for s in os.environ.get("HB_PROJ", "").split(",") if s]
    for name, N, K, resid in SHAPES:
        if only and name not in only:
            continue
        w = ((torch.rand(N, K, device=dev) * 2 - 1) * K ** -0.5).to(torch.bfloat16)
        for M in Ms:
            x = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
            r = (torch.rand(M, N, device=dev) * 2 - 1).to(torch.bfloat16)
            out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            t0 = time.time()
            cands = ops.hblt_candidates(M, N, K, resid)
            heur = cands[:1]
            screen = {}
            for c in cands:
                if ops.hblt_mm(x, w, c, out, resid=r if resid else None) is None:
                    continue
                screen[c] = timed(lambda c=c: ops.hblt_mm(x, w, c, out, resid=r if resid else None), 3)
            screen_s = time.time() - t0
            best8 = sorted(screen, key=screen.get)[:8]
            fns = {f"sol{c}": (lambda c=c: ops.hblt_mm(x, w, c, out, resid=r if resid else None)) for c in best8}
            rr = r.clone()
            fns["torch"] = (lambda: rr.addmm_(x, w.t())) if resid else (lambda: torch.nn.functional.linear(x, w))
            for tr, mi in ((256, 0), (256, 16), (224, 0), (192, 0), (192, 32), (160, 0)):
                fns[f"pf{tr}/{mi}"] = (lambda tr=tr, mi=mi: ops.gemm_pf(x, w, 2 if resid else 0, out, mi,
                                                                        resid=r if resid else None, trows=tr))
            ts = {k: [] for k in fns}
            for _ in range(5):
                for k, fn in fns.items():
                    ts[k].append(timed(fn))
            med = {k: round(statistics.median(v), 2) for k, v in ts.items()}
            best = min((k for k in med if k.startswith("sol")), key=med.get)
            # correctness of the best solution against fp32
            ref = x.float() @ w.float().t() + (r.float() if resid else 0)
            got = ops.hblt_mm(x, w, int(best[3:]), None, resid=r if resid else None)
            err = ((got.float() - ref).abs().max() / ref.abs().max()).item()
            pf_best = min((k for k in med if k.startswith("pf")), key=med.get)
            fl = 2.0 * M * N * K
            print(json.dumps({"proj": name, "M": M, "N": N, "K": K, "resid": resid, "candidates": len(cands),
                              "supported_run": len(screen), "screen_s": round(screen_s, 1),
                              "heuristic_top": heur, "us": med, "best": best,
                              "best_kernel": ops.ext().hblt_kernel_name(int(best[3:]))[:120],
                              "best_TF": round(fl / med[best] / 1e6, 1), "torch_TF": round(fl / med["torch"] / 1e6, 1),
                              "best_vs_torch": round(med["torch"] / med[best], 3), "pf_best": pf_best,
                              "best_vs_pf": round(med[pf_best] / med[best], 3), "rel_err": round(err, 5)}), flush=True)


if __name__ == "__main__":
    main()
