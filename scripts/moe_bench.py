"""Mixtral-8x7B MoE layer on one GPU: grouped-GEMM path vs per-expert hipBLASLt loop."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import torch  # noqa: E402

from mxserve import ops  # noqa: E402
from mxserve.ops import moe  # noqa: E402


def timeit(fn, iters=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    dev = torch.device("cuda:0")
    H, I, E, K = 4096, 14336, 8, 2
    w13 = torch.randn(E, 2 * I, H, device=dev, dtype=torch.bfloat16) * 0.02
    w2 = torch.randn(E, H, I, device=dev, dtype=torch.bfloat16) * 0.02
    for T in (64, 256, 2048, 8192):  # fused_experts switches to the loop above GROUPED_MAX_TOKENS
        x = torch.randn(T, H, device=dev, dtype=torch.bfloat16)
        tw, tid = ops.moe_topk_softmax(torch.randn(T, E, device=dev, dtype=torch.bfloat16), K)
        flops = 2 * T * K * (2 * I * H + H * I)
        cap = moe.GROUPED_MAX_TOKENS
        moe.GROUPED_MAX_TOKENS = 1 << 30  # time the grouped kernel at every T
        tg = timeit(lambda: moe.fused_experts(x, w13, w2, tw, tid, 0))
        moe.GROUPED_MAX_TOKENS = cap
        tl = timeit(lambda: moe._fused_experts_loop(x, w13, w2, tw, tid, 0))
        print(json.dumps({"op": "moe_layer", "T": T, "grouped_ms": round(tg, 4), "loop_ms": round(tl, 4),
                          "grouped_TFLOPs": round(flops / tg / 1e9, 1), "loop_TFLOPs": round(flops / tl / 1e9, 1)}),
              flush=True)


if __name__ == "__main__":
    main()
