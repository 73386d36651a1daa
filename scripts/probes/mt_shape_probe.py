"""Kernel durations of the decode GEMM forms at one projection shape, for rocprofv3 --kernel-trace:
hipBLASLt and the medium-M (mt) kernel at several split-K factors, each on 8 cold weight copies.
  python scripts/probes/mt_shape_probe.py M N K [cfg;cfg...]   (cfg = comma list, e.g. mt,4,2,1,2,4)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from mxserve.ops import decode_gemm as dg  # noqa: E402

M, N, K = (int(v) for v in sys.argv[1:4])
cfgs = [tuple(int(x) if x.lstrip("-").isdigit() else x for x in c.split(",")) for c in sys.argv[4].split(";")] \
    if len(sys.argv) > 4 else [("mt", 4, 2, 1, 2, s) for s in (1, 2, 4, 8)]
dev = torch.device("cuda:0")
dg.TABLE.part = torch.empty(16 * 448 * 16384, dtype=torch.float32, device=dev)
ws = [(torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16) for _ in range(8)]
x = torch.randn(M, K, device=dev).to(torch.bfloat16)
out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
for rep in range(3):
    for w in ws:
        torch.nn.functional.linear(x, w)
    torch.cuda.synchronize()
    for cfg in cfgs:
        for w in ws:
            dg.TABLE.run(out, x, w, cfg, 0)
        torch.cuda.synchronize()
print("done", cfgs)
