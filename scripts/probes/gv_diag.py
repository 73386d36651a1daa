"""Per-configuration max error of gemv_stream against fp32 (debug aid)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from mxserve.ops import decode_gemm  # noqa: E402

gpu = "cuda:0"
for (N, K, epi) in [(1280, 8192, 0), (8192, 1024, 0), (7168, 8192, 1), (3072, 2048, 0)]:
    for M in (1, 4):
        x = torch.randn(M, K, device=gpu, dtype=torch.bfloat16)
        w = (torch.randn(N, K, device=gpu) * K ** -0.5).to(torch.bfloat16)
        y = x.float() @ w.float().t()
        want = torch.nn.functional.silu(y[:, :N // 2]) * y[:, N // 2:] if epi else y
        for cfg in decode_gemm.gv_candidates(M, N, K, epi):
            out = torch.full(want.shape, float("nan"), device=gpu, dtype=torch.bfloat16)
            ok = decode_gemm.TABLE.run(out, x, w, cfg, epi)
            err = (out.float() - want).abs()
            bad = (err > 0.02 + 0.02 * want.abs())
            idx = bad.nonzero()[:4].tolist()
            print(N, K, epi, M, cfg, ok, "maxerr", round(err.max().item(), 4), "bad", int(bad.sum()), idx,
                  "nan", int(torch.isnan(out.float()).sum()), flush=True)
