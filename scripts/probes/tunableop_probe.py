"""hipBLASLt's default solution vs PyTorch TunableOp's pick (every hipBLASLt / rocBLAS solution timed,
rotating buffers so the weights are not cache-resident) for the prefill projections the packaged
table leaves on hipBLASLt: qkv (F.linear) and o / down (addmm_ into the residual), Llama-3.2-1B, at
the row buckets of the headline's mixed steps.  Writes the TunableOp results CSV to argv[1]."""
import json
import os
import sys

import torch

F = torch.nn.functional
out_csv = sys.argv[1]
dev = torch.device("cuda:0")
shapes = {"qkv": (3072, 2048, 0), "o": (2048, 2048, 2), "down": (2048, 8192, 2)}
Ms = [4096, 5120, 6144, 6592]


def timed(fn, iters=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3 / iters)
    return sorted(ts)[2]


cases = []
for name, (N, K, epi) in shapes.items():
    w = (torch.randn(N, K, device=dev) * K ** -0.5).to(torch.bfloat16)
    for M in Ms:
        x = torch.randn(M, K, device=dev).to(torch.bfloat16)
        r = torch.randn(M, N, device=dev).to(torch.bfloat16)
        fn = (lambda x=x, w=w, r=r: r.addmm_(x, w.t())) if epi == 2 else (lambda x=x, w=w: F.linear(x, w))
        cases.append((name, M, fn))
base = {(n, M): timed(fn) for n, M, fn in cases}
torch.cuda.tunable.enable(True)
torch.cuda.tunable.tuning_enable(True)
torch.cuda.tunable.set_filename(out_csv, insert_device_ordinal=False)
torch.cuda.tunable.set_max_tuning_duration(200)
torch.cuda.tunable.set_rotating_buffer_size(512)
for n, M, fn in cases:
    fn()  # tunes this shape
torch.cuda.synchronize()
torch.cuda.tunable.tuning_enable(False)
for n, M, fn in cases:
    t = timed(fn)
    print(json.dumps({"proj": n, "M": M, "hipblaslt_default_us": round(base[(n, M)], 2), "tunableop_us": round(t, 2),
                      "speedup": round(base[(n, M)] / t, 3)}), flush=True)
print(json.dumps({"results": [list(map(str, r)) for r in torch.cuda.tunable.get_results()]}), flush=True)
