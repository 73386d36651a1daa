#!/usr/bin/env python3
"""Paged prefill attention alone (csrc/kernels/attention_prefill.hip v3): causal, fresh sequences of
`per` tokens each (the bench's 8192-token chunk = 2 x 4096), Llama-3.2-1B heads (32 q / 8 kv, D 64)
and Llama-3-8B-like D 128; one JSON line per case with ms and TFLOP/s (causal half counted).
PA_VARS=0,2,6 times the softmax variants of the v3 kernel (version 0x100 | VAR, G = 4 only) round-robin
on the same inputs and reports each one's max |diff| against the first; -1 is the default launch (which
picks the split variant 128 for small grids)."""
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from mxserve import ops
    dev = torch.device("cuda:0")
    cases = ((64, 32, 8, 2, 4096), (64, 32, 8, 1, 8192), (128, 32, 8, 2, 4096))
    if os.environ.get("PA_CASE"):  # one case (counter passes): index into cases
        cases = (cases[int(os.environ["PA_CASE"])],)
    if os.environ.get("PA_SHAPES"):  # Llama-3.2-1B heads at NxL[xD] shapes (D 64 default), e.g. "1x4096,4x2048x128"
        cases = tuple((int((c.split("x") + ["64"])[2]), 32, 8, int(c.split("x")[0]), int(c.split("x")[1]))
                      for c in os.environ["PA_SHAPES"].split(","))
    for D, hq, hkv, nseq, per in cases:
        T = nseq * per
        pb = math.ceil(per / 16)
        bt = torch.arange(nseq * pb, device=dev, dtype=torch.int32).view(nseq, pb)
        kv = (torch.randn(nseq * pb, 2, hkv, 16, D, device=dev) * 0.5).to(torch.bfloat16)
        q = torch.randn(T, hq, D, dtype=torch.bfloat16, device=dev)
        qsl = torch.tensor([i * per for i in range(nseq + 1)], dtype=torch.int32, device=dev)
        sl = torch.full((nseq,), per, dtype=torch.int32, device=dev)
        variants = [int(v) for v in os.environ.get("PA_VARS", "").split(",") if v != ""] or [None]
        flops = 4 * nseq * per * per / 2 * D * hq
        ref_out, times = None, {v: [] for v in variants}
        for rnd in range(3):
            for v in variants:
                ver = 0 if v is None else (3 if v < 0 else 0x100 + v)  # -1: the default launch (split gate)
                fn = lambda: ops.paged_attention_prefill(q, kv, bt, qsl, sl, D ** -0.5, per, version=ver)  # noqa: E731
                for _ in range(3):
                    out = fn()
                if rnd == 0:
                    if ref_out is None:
                        ref_out = out.float()
                    err = (out.float() - ref_out).abs().max().item()
                    if err > 0.05 or not torch.isfinite(out).all():
                        print(json.dumps({"D": D, "var": v, "error": "mismatch", "max_diff": err}), flush=True)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(20):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                times[v].append(e0.elapsed_time(e1) / 20)
        for v in variants:
            ms = sorted(times[v])[1]
            print(json.dumps({"D": D, "hq": hq, "hkv": hkv, "seqs": nseq, "per_seq": per, "var": v, "ms": round(ms, 4),
                              "TFLOPs": round(flops / ms / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
