#!/usr/bin/env python3
"""Prefill layer projections with the RMSNorm / residual add fused into gemm_pf (row-scale consumer +
residual epilogue) vs the current chain, Llama-3.2-1B shapes, per row count (argv, default 2048 4096
6400 8192).  Interleaved rounds in one process; JSON lines to stdout and gpurun_out/pf_fused_probe.jsonl.

current (per layer, projections + norms only):
  o: linear -> add+RMSNorm kernel -> gate_up (gemm_pf SwiGLU or hipBLASLt + silu_mul) -> down: linear
  -> add+RMSNorm kernel -> qkv: linear
fused:
  o: gemm_pf epi 2 (residual in place) -> gate_up: gemm_pf SwiGLU + row scale -> down: gemm_pf epi 2
  -> qkv: gemm_pf + row scale
Also per-op candidates (min_iters 0/8/16/32; o/down as hipBLASLt addmm_ with beta = 1)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    from mxserve import ops
    dev = torch.device("cuda:0")
    H, I, NQKV = 2048, 8192, 3072
    eps = 1e-5
    g = torch.Generator(device="cuda").manual_seed(0)

    def W(n, k):
        return (torch.randn(n, k, device=dev, generator=g) * k ** -0.5).to(torch.bfloat16)
    wqkv, wo, wgu, wd = W(NQKV, H), W(H, H), W(2 * I, H), W(H, I)
    g_in = (1 + 0.1 * torch.randn(H, device=dev, generator=g)).to(torch.bfloat16)
    g_post = (1 + 0.1 * torch.randn(H, device=dev, generator=g)).to(torch.bfloat16)
    wqkv_f, wgu_f = ops.fold_norm_weight(wqkv, g_in), ops.fold_norm_weight(wgu, g_post)
    rows = []
    mis = [int(v) for v in os.environ.get("PFP_MI", "0,8,16,32").split(",")]
    for M in (int(a) for a in (sys.argv[1:] or ["2048", "4096", "6400", "8192"])):
        a = torch.randn(M, H, device=dev, generator=g).to(torch.bfloat16)
        m_in = torch.randn(M, I, device=dev, generator=g).to(torch.bfloat16)
        r0 = (torch.randn(M, H, device=dev, generator=g) * 2).to(torch.bfloat16)
        r = r0.clone()
        fns = {
            # current chain pieces
            "cur_o": lambda: ops.linear(a, wo),
            "cur_addnorm": lambda: ops.fused_add_rms_norm(a, r, g_post, eps),
            "cur_gate_up": lambda: ops.gate_up_silu(a, wgu),
            "cur_down": lambda: ops.linear(m_in, wd),
            "cur_qkv": lambda: ops.linear(a, wqkv),
            "norm_only": lambda: ops.rms_norm(r, g_in, eps),
            "addmm_o": lambda: r.addmm_(a, wo.t()),
            "addmm_down": lambda: r.addmm_(m_in, wd.t()),
        }
        for mi in mis:
            fns[f"pf_o_resid/{mi}"] = lambda mi=mi: ops.gemm_pf(a, wo, 2, r, mi, resid=r)
            fns[f"pf_down_resid/{mi}"] = lambda mi=mi: ops.gemm_pf(m_in, wd, 2, r, mi, resid=r)
            fns[f"pf_gu_rs/{mi}"] = lambda mi=mi: ops.gemm_pf(r, wgu_f, 1, None, mi, row_scale=True, eps=eps)
            fns[f"pf_qkv_rs/{mi}"] = lambda mi=mi: ops.gemm_pf(r, wqkv_f, 0, None, mi, row_scale=True, eps=eps)
            fns[f"pf_qkv/{mi}"] = lambda mi=mi: ops.gemm_pf(a, wqkv, 0, None, mi)
            fns[f"pf_o/{mi}"] = lambda mi=mi: ops.gemm_pf(a, wo, 0, None, mi)
            fns[f"pf_down/{mi}"] = lambda mi=mi: ops.gemm_pf(m_in, wd, 0, None, mi)
        ts = {k: [] for k in fns}
        for _ in range(3):
            for k, fn in fns.items():
                r.copy_(r0)
                ts[k].append(timed(fn))
        t = {k: round(min(v), 2) for k, v in ts.items()}

        def best(prefix):
            c = {k: v for k, v in t.items() if k.startswith(prefix + "/")}
            k = min(c, key=c.get)
            return k, c[k]
        cur = t["cur_o"] + 2 * t["cur_addnorm"] + t["cur_gate_up"] + t["cur_down"] + t["cur_qkv"]
        parts = {p: best(p) for p in ("pf_o_resid", "pf_down_resid", "pf_gu_rs", "pf_qkv_rs")}
        # best mix: each consumer picks fused or (norm pass + current op); each residual producer picks
        # gemm_pf epi 2 or hipBLASLt addmm_
        mix = (min(parts["pf_o_resid"][1], t["addmm_o"]) + min(parts["pf_down_resid"][1], t["addmm_down"]) +
               min(parts["pf_gu_rs"][1], t["norm_only"] + t["cur_gate_up"]) +
               min(parts["pf_qkv_rs"][1], t["norm_only"] + t["cur_qkv"]))
        fused = sum(v[1] for v in parts.values())
        row = {"M": M, "current_us": round(cur, 2), "fused_us": round(fused, 2), "best_mix_us": round(mix, 2),
               "speedup_fused": round(cur / fused, 3), "speedup_mix": round(cur / mix, 3),
               "best": {p: v[0] for p, v in parts.items()}, "times_us": t}
        # correctness spot check of the fused chain against the current one (one layer's projections)
        r.copy_(r0)
        h, _ = ops.fused_add_rms_norm(ops.linear(a, wo), r, g_post, eps)
        y_cur = ops.gate_up_silu(h, wgu)
        r2 = r0.clone()
        ops.gemm_pf(a, wo, 2, r2, 16, resid=r2)
        y_f = ops.gemm_pf(r2, wgu_f, 1, None, 16, row_scale=True, eps=eps)
        row["max_rel_err_gate_up"] = round(float((y_f.float() - y_cur.float()).abs().max() /
                                                 y_cur.float().abs().max()), 5)
        row["resid_equal"] = bool(torch.allclose(r2.float(), r.float(), atol=0.05, rtol=0.02))
        rows.append(row)
        print(json.dumps(row), flush=True)
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/pf_fused_probe.jsonl", "w") as f:
        for r_ in rows:
            f.write(json.dumps(r_) + "\n")


if __name__ == "__main__":
    main()
