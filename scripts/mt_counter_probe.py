#!/usr/bin/env python3
"""One decode projection on the mt kernel (or hipBLASLt), launched back to back for PMC counter
passes: `rocprofv3 --pmc <counters> -- python3 scripts/mt_counter_probe.py PROJ M CFG`.
PROJ: qkv | o | gate_up | down (Llama-3.2-1B shapes); CFG: lib | mt,wm,wn,mr,wnf,sk[,order]."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
SHAPES = {"qkv": (3072, 2048, 0), "o": (2048, 2048, 0), "gate_up": (16384, 2048, 1), "down": (2048, 8192, 0)}


def main():
    from mxserve.ops import decode_gemm as dg, silu_mul
    proj, M, cfg = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    N, K, epi = SHAPES[proj]
    dev = torch.device("cuda:0")
    w = ((torch.rand(N, K, device=dev) * 2 - 1) * K ** -0.5).to(torch.bfloat16)
    x = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
    out = torch.empty(M, N // 2 if epi else N, device=dev, dtype=torch.bfloat16)
    dg.TABLE.part = torch.empty(8 * M * N, dtype=torch.float32, device=dev)
    if cfg == "lib":
        fn = (lambda: silu_mul(torch.nn.functional.linear(x, w))) if epi else (lambda: torch.nn.functional.linear(x, w))
    else:
        parts = cfg.split(",")
        c = ("mt",) + tuple(int(v) for v in parts[1:])
        assert dg.TABLE.run(out, x, w, c, epi), c
        fn = lambda: dg.TABLE.run(out, x, w, c, epi)  # noqa: E731
    for _ in range(200):
        fn()
    torch.cuda.synchronize()
    print("done", proj, M, cfg)


if __name__ == "__main__":
    main()
