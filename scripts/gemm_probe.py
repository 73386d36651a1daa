#!/usr/bin/env python3
"""gemm_pf (csrc/kernels/gemm_pf.hip) at several stream-K segment lengths (GB_PF) vs hipBLASLt (torch
F.linear) at the Llama-3.2-1B projections (GB_SHAPES), random operands, interleaved rounds in one
process (cdna_hip_programming.md §5.4 rule 24).  gate_up compares the fused SwiGLU epilogue with
hipBLASLt + the SiLU*mul kernel.  JSON lines.  (The earlier gemm_big kernel and its ping-pong variants
that led to gemm_pf were removed in round 4; profiles/r4/gemm_pingpong_v6_vs_hipblaslt.jsonl.)"""
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
    return s.elapsed_time(e) / iters * 1e3  # us


def main():
    from mxserve import ops
    dev = torch.device("cuda:0")
    out = []
    shapes = {"qkv": (3072, 2048), "o": (2048, 2048), "gate_up": (16384, 2048), "down": (2048, 8192),
              "lm_head": (128256, 2048)}
    only = [s for s in os.environ.get("GB_SHAPES", "qkv,o,gate_up,down").split(",") if s]
    shapes = {k: v for k, v in shapes.items() if k in only}
    for M in (int(a) for a in (sys.argv[1:] or ["8192", "4096", "2048"])):
        for name, (N, K) in shapes.items():
            x = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
            w = ((torch.rand(N, K, device=dev) * 2 - 1) * K ** -0.5).to(torch.bfloat16)
            swiglu = name == "gate_up"
            y = torch.empty(M, N // 2 if swiglu else N, device=dev, dtype=torch.bfloat16)
            if swiglu:
                lib = lambda: ops.silu_mul(torch.nn.functional.linear(x, w))  # noqa: E731
            else:
                lib = lambda: torch.nn.functional.linear(x, w)  # noqa: E731
            ref = lib()
            fl = 2 * M * N * K
            row = {"proj": name, "M": M, "N": N, "K": K, "fused_swiglu": swiglu}
            fns = {"hipblaslt": lib}
            for mi in [int(v) for v in os.environ.get("GB_PF", "0,16").split(",") if v]:
                fns[f"pf{mi}"] = (lambda mi=mi: ops.gemm_pf(x, w, 1 if swiglu else 0, y, mi))
                assert fns[f"pf{mi}"]() is not None
                row[f"pf{mi}_rel_err"] = round(float((y.float() - ref.float()).abs().max() / ref.float().abs().max()), 5)
            ts = {k: [] for k in fns}
            for _ in range(3):
                for k, fn in fns.items():
                    ts[k].append(timed(fn))
            for k in fns:
                row[f"{k}_us"] = round(min(ts[k]), 2)
                row[f"{k}_TF"] = round(fl / min(ts[k]) / 1e6, 1)
            out.append(row)
            print(json.dumps(row), flush=True)
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/gemm_probe.jsonl", "w") as f:
        for r in out:
            f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
