"""Row-stream GEMV (gemm_decode.hip gemv_stream_kernel) vs hipBLASLt and the table's other forms at
M = 1-4: Llama-3-70B TP-8 shard shapes and the Llama-3.2-1B projections, cold weights (copies cycled
past the Infinity Cache), hipGraph-timed.  JSON lines with microseconds and weight TB/s."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from mxserve import ops  # noqa: E402
from mxserve.ops import decode_gemm as dg  # noqa: E402

dev = torch.device("cuda:0")
F = torch.nn.functional
shapes = {"tp8_qkv": (1280, 8192, 0), "tp8_o": (8192, 1024, 0), "tp8_gate_up": (7168, 8192, 1),
          "tp8_down": (8192, 3584, 0), "1b_qkv": (3072, 2048, 0), "1b_gate_up": (16384, 2048, 1),
          "1b_down": (2048, 8192, 0)}
Ms = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "1,4").split(",")]
dg.TABLE.part = torch.empty(64 * 64 * 16384, dtype=torch.float32, device=dev)
for name, (N, K, epi) in shapes.items():
    ws = dg.weight_copies((torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16))
    for M in Ms:
        x = torch.randn(M, K, device=dev).to(torch.bfloat16)
        out = torch.empty(M, N // 2 if epi else N, device=dev, dtype=torch.bfloat16)
        base = (lambda i: ops.silu_mul(F.linear(x, ws[i % len(ws)]))) if epi else (lambda i: F.linear(x, ws[i % len(ws)]))
        res = [("hipblaslt", dg._graph_time(base))]
        for cfg in dg.candidates(M, N, K, epi):
            if cfg[0] in ("gv", "sk"):
                res.append((cfg, dg._graph_time(lambda i, c=cfg: dg.TABLE.run(out, x, ws[i % len(ws)], c, epi))))
        res.sort(key=lambda r: r[1])
        byts = N * K * 2
        print(json.dumps({"shape": name, "M": M, "best": [(str(c), round(t, 2), round(byts / t / 1e6, 2)) for c, t in res[:4]],
                          "hipblaslt_us": round(dict((str(c), t) for c, t in res)["hipblaslt"], 2)}), flush=True)
