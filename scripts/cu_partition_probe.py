#!/usr/bin/env python3
"""Can a bandwidth-bound decode-attention stream and a compute-bound prefill stream share one MI355X
on disjoint CU sets (hipExtStreamCreateWithCUMask) and finish sooner than back to back?

Plain concurrent streams did not overlap (profiles/r3/overlap_probe_decode_vs_prefill_streams.jsonl:
each kernel fills the chip, 0.91-1.04x).  Here stream A runs Llama-3.2-1B decode attention (B = 384,
ctx 4250, one layer, ~3.3 GB of KV per call) on X CUs and stream B the prefill MLP GEMMs of an
8192-token chunk (gate_up with SiLU on gemm_pf, down on hipBLASLt) on the other 256 - X.  Per X:
each side alone on its mask, then both together; speedup = (A + B on the full chip) / together.
Mask layouts: xcd (X / 8 CUs of every 32-CU block of the mask) and low (the first X bits).
"""
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def masks(X: int, ncu: int, layout: str):
    words = (ncu + 31) // 32
    a = [0] * words
    if layout == "xcd":  # X / 8 CUs out of every block of ncu / 8 bits
        per = ncu // 8
        k = X // 8
        for x in range(8):
            for j in range(k):
                c = x * per + j
                a[c // 32] |= 1 << (c % 32)
    else:
        for c in range(X):
            a[c // 32] |= 1 << (c % 32)
    full = [(1 << 32) - 1] * words
    b = [f & ~w & 0xFFFFFFFF for f, w in zip(full, a)]
    return a, b


def main():
    from mxserve import ops
    ext = ops.ext()
    dev = torch.device("cuda:0")
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    # --- A: decode attention, one layer
    B, ctx, D, hkv, G = 384, 4250, 64, 8, 4
    nbps = math.ceil((ctx + 1) / 16)
    nb = B * nbps
    kv = (torch.randn(nb, 2, hkv, 16, D, device=dev) * 0.3).to(torch.bfloat16)
    bt = torch.randperm(nb, device=dev).view(B, nbps).to(torch.int32)
    sl = torch.full((B,), ctx + 1, dtype=torch.int32, device=dev)
    q = torch.randn(B, hkv * G, D, dtype=torch.bfloat16, device=dev)
    oa = torch.empty_like(q)
    fa = lambda: ops.paged_attention_decode(q, kv, bt, sl, D ** -0.5, ctx + 1, out=oa)  # noqa: E731
    # --- B: prefill MLP of an 8192-token chunk
    M = 8192
    x = (torch.randn(M, 2048, device=dev) * 0.5).to(torch.bfloat16)
    wgu = (torch.randn(16384, 2048, device=dev) * 2048 ** -0.5).to(torch.bfloat16)
    wd = (torch.randn(2048, 8192, device=dev) * 8192 ** -0.5).to(torch.bfloat16)
    act = torch.empty(M, 8192, dtype=torch.bfloat16, device=dev)

    def fb():
        ops.gemm_pf(x, wgu, 1, act, 0)
        torch.nn.functional.linear(act, wd)

    def timed(pairs, n=10):
        """pairs: [(stream, fn, calls)] all launched together; returns wall ms and each stream's ms."""
        start = torch.cuda.Event(enable_timing=True)
        ends = []
        torch.cuda.synchronize()
        start.record()
        for s, fn, calls in pairs:
            s.wait_event(start)
            with torch.cuda.stream(s):
                for _ in range(calls):
                    fn()
                e = torch.cuda.Event(enable_timing=True)
                e.record()
            ends.append(e)
        torch.cuda.synchronize()
        return [start.elapsed_time(e) for e in ends]

    full = torch.cuda.Stream()
    for _ in range(2):
        timed([(full, fa, 3)])
        timed([(full, fb, 3)])
    NA, NB = 12, 6
    ta = timed([(full, fa, NA)])[0]
    tb = timed([(full, fb, NB)])[0]
    print(json.dumps({"op": "full_chip", "attn_ms_per_call": round(ta / NA, 4), "mlp_ms_per_call": round(tb / NB, 4),
                      "attn_TBps": round(B * (ctx + 1) * hkv * D * 4 / (ta / NA) / 1e9, 2)}), flush=True)
    streams = []
    for layout in ("xcd", "low"):
        for X in (64, 96, 128, 160, 192):
            ma, mb = masks(X, ncu, layout)
            pa, pb = ext.cu_mask_stream(ma), ext.cu_mask_stream(mb)
            streams += [pa, pb]
            sa, sb = torch.cuda.ExternalStream(pa), torch.cuda.ExternalStream(pb)
            timed([(sa, fa, 2)])
            timed([(sb, fb, 2)])
            a_alone = timed([(sa, fa, NA)])[0]
            b_alone = timed([(sb, fb, NB)])[0]
            both = timed([(sa, fa, NA), (sb, fb, NB)])
            wall = max(both)
            row = {"op": "partition", "layout": layout, "attn_cus": X, "mlp_cus": ncu - X,
                   "attn_alone_ms": round(a_alone, 3), "mlp_alone_ms": round(b_alone, 3),
                   "attn_together_ms": round(both[0], 3), "mlp_together_ms": round(both[1], 3),
                   "serial_full_chip_ms": round(ta + tb, 3), "together_ms": round(wall, 3),
                   "speedup_vs_serial": round((ta + tb) / wall, 3),
                   "attn_TBps_alone": round(B * (ctx + 1) * hkv * D * 4 / (a_alone / NA) / 1e9, 2)}
            print(json.dumps(row), flush=True)
    torch.cuda.synchronize()
    for p in streams:
        ext.stream_destroy(p)


if __name__ == "__main__":
    main()
