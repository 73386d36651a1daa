#!/usr/bin/env python3
"""Mixed-step attention: the decode kernel (HBM-bound: the whole KV of the running set) and the prefill
kernel (MFMA-bound: one new 4k-token chunk) of ONE layer, back to back on one stream vs concurrently on
two streams (forked and joined with events, the way a mixed step would issue them).  Llama-3.2-1B
layer shapes, random data.  JSON lines: mode, ms per layer (20 iterations, after warmup)."""
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from mxserve import ops
    dev = torch.device("cuda:0")
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 192
    ctx = int(sys.argv[2]) if len(sys.argv) > 2 else 4000
    T = int(sys.argv[3]) if len(sys.argv) > 3 else 4000
    nh, nkv, D = 32, 8, 64
    nbps = math.ceil((ctx + 1) / 16)
    pb = math.ceil(T / 16)
    nb = B * nbps + pb + 16
    kv = torch.randn(nb, 2, nkv, 16, D, dtype=torch.bfloat16, device=dev) * 0.1
    bt = torch.randperm(B * nbps, device=dev)[:B * nbps].view(B, nbps).to(torch.int32)
    sl = torch.full((B,), ctx + 1, dtype=torch.int32, device=dev)
    qd = torch.randn(B, nh, D, dtype=torch.bfloat16, device=dev)
    od = torch.empty_like(qd)
    bt2 = (B * nbps + torch.arange(pb, device=dev, dtype=torch.int32)).view(1, pb)
    qsl = torch.tensor([0, T], dtype=torch.int32, device=dev)
    sl2 = torch.tensor([T], dtype=torch.int32, device=dev)
    qp = torch.randn(T, nh, D, dtype=torch.bfloat16, device=dev)
    op = torch.empty_like(qp)

    dec = lambda: ops.paged_attention_decode(qd, kv, bt, sl, 0.125, 8192, out=od)  # noqa: E731
    pre = lambda: ops.paged_attention_prefill(qp, kv, bt2, qsl, sl2, 0.125, T, out=op)  # noqa: E731
    side = torch.cuda.Stream()
    main_s = torch.cuda.current_stream()

    def both_concurrent():
        ev = torch.cuda.Event()
        ev.record(main_s)
        side.wait_event(ev)
        with torch.cuda.stream(side):
            dec()
        pre()
        ev2 = torch.cuda.Event()
        ev2.record(side)
        main_s.wait_event(ev2)

    def both_serial():
        dec()
        pre()

    def timeit(fn, iters=20):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / iters

    res = {"B": B, "ctx": ctx, "T": T}
    for name, fn in (("decode", dec), ("prefill", pre), ("serial", both_serial), ("concurrent", both_concurrent),
                     ("serial2", both_serial), ("concurrent2", both_concurrent)):
        res[name + "_ms"] = round(timeit(fn), 4)
    ref = od.clone(), op.clone()
    both_concurrent()
    torch.cuda.synchronize()
    res["concurrent_matches_serial"] = bool(torch.equal(ref[0], od) and torch.equal(ref[1], op))
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
