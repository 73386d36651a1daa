#!/usr/bin/env python3
"""Prefill K RoPE + paged K / V cache write (rope_kv_into_cache -> kv_rope_t16_kernel) at
Llama-3.2-1B shapes over chunk sizes, hipGraph-timed; JSON lines with us and the bytes' rate."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    from mxserve import ops
    from mxserve.ops import reference as ref
    dev = torch.device("cuda:0")
    hq, hkv, D = 32, 8, 64
    cs = ref.build_cos_sin_cache(D, 16384, 500000.0, None, device=dev)
    for T in (1024, 2400, 4000, 6144, 8192):
        nb = T // 16 + 64
        kv = torch.zeros(nb, 2, hkv, 16, D, device=dev, dtype=torch.bfloat16)
        qkv = torch.randn(T, (hq + 2 * hkv) * D, device=dev, dtype=torch.bfloat16)
        pos = torch.arange(T, device=dev) + 1000
        slots = torch.arange(T, device=dev) + 16 * 7
        fn = lambda: ops.rope_kv_into_cache(qkv, hq, hkv, D, pos, cs, kv, slots)  # noqa: E731
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(20):
                fn()
        ts = []
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            g.replay()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3 / 20)
        us = sorted(ts)[2]
        byts = T * hkv * D * 2 * 2 * 2  # K and V read + written
        print(json.dumps({"T": T, "us": round(us, 2), "TBps": round(byts / us / 1e6, 2)}), flush=True)


if __name__ == "__main__":
    main()
