"""Decode attention (Llama-3.2-1B: 8 kv heads, D 64, G 4) at the headline's running-set sizes with
context 4000-4500 per sequence, one layer; the partition plan's workgroup floor comes from
MXS_DECODE_TARGET_WGS (read once per process, so run one process per setting).  JSON lines."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from mxserve import ops  # noqa: E402

dev = torch.device("cuda:0")
torch.manual_seed(0)
D, G, Hkv = 64, 4, 8
for B in [int(b) for b in os.environ.get("DP_BATCHES", "256,288,320,384,448").split(",")]:
    lens = torch.randint(4000, 4501, (B,), dtype=torch.int32)
    nb = [(int(l) + 15) // 16 for l in lens]
    mb = max(nb)
    tot = sum(nb)
    kv = (torch.randn(tot + 8, 2, Hkv, 16, D, device=dev) * 0.3).to(torch.bfloat16)
    perm = torch.randperm(tot, device=dev).to(torch.int32)
    bt = torch.zeros(B, mb, dtype=torch.int32, device=dev)
    o = 0
    for i, n in enumerate(nb):
        bt[i, :n] = perm[o:o + n]
        o += n
    q = torch.randn(B, Hkv * G, D, device=dev, dtype=torch.bfloat16)
    sl = lens.to(dev)
    fn = lambda: ops.paged_attention_decode(q, kv, bt, sl, D ** -0.5, 8192)  # noqa: E731
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / 10)
    ms = sorted(ts)[2]
    byts = int(lens.sum()) * Hkv * D * 2 * 2
    print(json.dumps({"target_wgs": int(os.environ.get("MXS_DECODE_TARGET_WGS", "2048")), "B": B,
                      "us": round(ms * 1e3, 1), "TBps": round(byts / ms / 1e9, 3)}), flush=True)
