#!/usr/bin/env python3
"""Do decode attention (HBM-bound) and prefill attention (MFMA/VALU-bound) of ONE mixed step overlap
when launched on two HIP streams?

A mixed engine step runs, per layer, the decode rows' paged attention (B=256 at ctx 4000: ~2 GB of
KV, ~0.33 ms) and then the prefill chunk's causal attention (a few thousand tokens: ~0.1-0.2 ms at
~700 TF) back to back.  The earlier probe (scripts/overlap_probe.py) paired decode attention with a
prefill GEMM, whose 256 workgroups hold whole CUs; prefill ATTENTION workgroups are smaller, so the
decode workgroups may fill in beside them.  Prints JSON lines: serial (one stream) vs concurrent
(prefill launched first on stream P, decode on stream D), for a few chunk shapes."""
from __future__ import annotations

import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def ev():
    return torch.cuda.Event(enable_timing=True)


def timed(fn, iters=20, warmup=3) -> float:
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    s, e = ev(), ev()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    from mxserve import ops
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    nkv, nh, D, bs = 8, 32, 64, 16
    B, ctx = 256, 4000
    nbps = math.ceil((ctx + 1) / bs)
    shapes = [(1, 3072, 0), (2, 2048, 0), (1, 4096, 0), (1, 2048, 2000), (3, 2730, 0)]
    maxp = max(n * math.ceil((t + c) / bs) for n, t, c in shapes)
    nb = B * nbps + maxp + 16
    kv = torch.randn(nb, 2, nkv, bs, D, dtype=torch.bfloat16, device=dev) * 0.1
    bt = torch.randperm(B * nbps, device=dev).view(B, nbps).to(torch.int32)
    sl = torch.full((B,), ctx + 1, dtype=torch.int32, device=dev)
    qd = torch.randn(B, nh, D, dtype=torch.bfloat16, device=dev)
    od = torch.empty_like(qd)
    dec = lambda: ops.paged_attention_decode(qd, kv, bt, sl, 0.125, 8192, out=od)  # noqa: E731
    t_dec = timed(dec)
    print(json.dumps({"op": "decode_attn", "B": B, "ctx": ctx, "ms": round(t_dec, 4)}), flush=True)
    sd, sp = torch.cuda.Stream(), torch.cuda.Stream()
    rows = []
    for n, t, c in shapes:
        per_blocks = math.ceil((t + c) / bs)
        btp = (B * nbps + torch.arange(n * per_blocks, device=dev)).view(n, per_blocks).to(torch.int32)
        qsl = torch.arange(0, n * t + 1, t, dtype=torch.int32, device=dev)
        slp = torch.full((n,), t + c, dtype=torch.int32, device=dev)
        qp = torch.randn(n * t, nh, D, dtype=torch.bfloat16, device=dev)
        op = torch.empty_like(qp)
        pre = lambda: ops.paged_attention_prefill(qp, kv, btp, qsl, slp, 0.125, t, out=op)  # noqa: E731
        t_pre = timed(pre)

        def serial():
            pre()
            dec()

        def conc():
            start = torch.cuda.current_stream()
            e0 = ev()
            e0.record(start)
            sp.wait_event(e0)
            sd.wait_event(e0)
            with torch.cuda.stream(sp):
                pre()
            with torch.cuda.stream(sd):
                dec()
            start.wait_stream(sp)
            start.wait_stream(sd)
        t_ser = timed(serial)
        t_con = timed(conc)
        t_con2 = timed(conc)
        flops = 4 * D * nh * n * (t * c + t * t / 2)
        row = {"op": "overlap", "seqs": n, "chunk": t, "prefix": c, "prefill_ms": round(t_pre, 4),
               "prefill_TF": round(flops / t_pre / 1e9, 1), "decode_ms": round(t_dec, 4),
               "serial_ms": round(t_ser, 4), "concurrent_ms": round(min(t_con, t_con2), 4),
               "saved_of_prefill": round((t_ser - min(t_con, t_con2)) / t_pre, 3)}
        rows.append(row)
        print(json.dumps(row), flush=True)
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/attn_overlap_probe.jsonl", "w") as f:
        for r in rows:
            f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
