#!/usr/bin/env python3
"""Decode-attention rate across GQA shapes and KV dtypes (one layer, hipGraph-free timing):
Llama-3.2-1B (D 64, G 4), Llama-3-8B (D 128, G 4), Qwen3-0.6B (D 128, G 2), Llama-3-70B TP8 shard
(D 128, G 8, one kv head per rank).  Prints one JSON line per case: ms and effective TB/s of KV."""
from __future__ import annotations

import json
import math

import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mxserve import ops  # noqa: E402

CASES = [  # name, D, G, Hkv, B
    ("llama1b", 64, 4, 8, 256),
    ("llama8b", 128, 4, 8, 128),
    ("qwen3_0.6b", 128, 2, 8, 256),
    ("llama70b_tp8", 128, 8, 1, 256),
]


def timeit(fn, iters=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


def main():
    dev = torch.device("cuda:0")
    ctx = 4000
    for name, D, G, hkv, B in CASES:
        nbps = math.ceil((ctx + 1) / 16)
        nb = B * nbps + 8
        kv = torch.randn(nb, 2, hkv, 16, D, dtype=torch.bfloat16, device=dev) * 0.3
        kv8 = (kv.float() * 8).to(torch.float8_e4m3fn).view(torch.uint8)
        bt = torch.randperm(nb - 8, device=dev)[:B * nbps].view(B, nbps).to(torch.int32)
        sl = torch.full((B,), ctx + 1, dtype=torch.int32, device=dev)
        q = torch.randn(B, hkv * G, D, dtype=torch.bfloat16, device=dev)
        sc = 1 / math.sqrt(D)
        kv_bytes = B * (ctx + 1) * hkv * D * 2
        for dt, cache, kw in (("bf16", kv, {}), ("fp8", kv8, {"k_scale": 1 / 8, "v_scale": 1 / 8})):
            for impl, iname in ((1, "valu_dot2"), (2, "mfma")):
                ms = timeit(lambda: ops.paged_attention_decode(q, cache, bt, sl, sc, ctx + 1, impl=impl, **kw))
                byts = kv_bytes * (2 if dt == "bf16" else 1)
                print(json.dumps({"case": name, "D": D, "G": G, "Hkv": hkv, "B": B, "ctx": ctx, "kv": dt,
                                  "impl": iname, "ms": round(ms, 4), "TBps": round(byts / ms / 1e9, 3)}), flush=True)
        del kv, kv8


if __name__ == "__main__":
    main()
