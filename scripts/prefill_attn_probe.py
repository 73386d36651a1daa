#!/usr/bin/env python3
"""Paged prefill attention alone (csrc/kernels/attention_prefill.hip v3): causal, fresh sequences of
`per` tokens each (the bench's 8192-token chunk = 2 x 4096), Llama-3.2-1B heads (32 q / 8 kv, D 64)
and Llama-3-8B-like D 128; one JSON line per case with ms and TFLOP/s (causal half counted)."""
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
    for D, hq, hkv, nseq, per in cases:
        T = nseq * per
        pb = math.ceil(per / 16)
        bt = torch.arange(nseq * pb, device=dev, dtype=torch.int32).view(nseq, pb)
        kv = (torch.randn(nseq * pb, 2, hkv, 16, D, device=dev) * 0.5).to(torch.bfloat16)
        q = torch.randn(T, hq, D, dtype=torch.bfloat16, device=dev)
        qsl = torch.tensor([i * per for i in range(nseq + 1)], dtype=torch.int32, device=dev)
        sl = torch.full((nseq,), per, dtype=torch.int32, device=dev)
        fn = lambda: ops.paged_attention_prefill(q, kv, bt, qsl, sl, D ** -0.5, per)  # noqa: E731
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 20
        flops = 4 * nseq * per * per / 2 * D * hq
        print(json.dumps({"D": D, "hq": hq, "hkv": hkv, "seqs": nseq, "per_seq": per, "ms": round(ms, 4),
                          "TFLOPs": round(flops / ms / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
