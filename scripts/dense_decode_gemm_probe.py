"""Decode-sized dense GEMMs of Llama-3.2-1B (M = batch rows): hipBLASLt vs the grouped MFMA GEMM
run as a one-expert GEMM (optionally split-K over fp32 slices, and with SiLU*mul fused for gate_up),
timed inside hipGraphs (launch gaps as in the engine)."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from mxserve import ops  # noqa: E402


def timeit_graph(fn, iters=20):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(10):
            fn()
    for _ in range(2):
        g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters / 10 * 1e3  # us per call


def main():
    dev = torch.device("cuda:0")
    shapes = {"qkv": (3072, 2048), "o": (2048, 2048), "gate_up": (16384, 2048), "down": (2048, 8192)}
    for M in (64, 128, 256):
        for name, (N, K) in shapes.items():
            x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
            w = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02
            w3 = w.unsqueeze(0)
            offs = torch.tensor([0, M], dtype=torch.int32, device=dev)
            r = {"M": M, "proj": name, "N": N, "K": K, "hipblaslt_us": timeit_graph(lambda: F.linear(x, w))}
            if name == "gate_up":
                h = torch.empty(M, N // 2, device=dev, dtype=torch.bfloat16)
                r["hipblaslt+silu_us"] = timeit_graph(lambda: ops.silu_mul(F.linear(x, w)))
                r["grouped_silu_us"] = timeit_graph(lambda: ops.ext().moe_grouped_gemm(h, x, w3, offs, True))
            y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            r["grouped_us"] = timeit_graph(lambda: ops.ext().moe_grouped_gemm(y, x, w3, offs, False))
            for sp in (2, 4, 8):
                if sp > K // 64:
                    continue
                part = torch.empty(sp, M, N, device=dev, dtype=torch.float32)
                r[f"grouped_split{sp}+sum_us"] = timeit_graph(
                    lambda: (ops.ext().moe_grouped_gemm(y, x, w3, offs, False, sp, part), part.sum(0)))
            print(json.dumps({k: (round(v, 2) if isinstance(v, float) else v) for k, v in r.items()}), flush=True)


if __name__ == "__main__":
    main()
