#!/usr/bin/env python3
"""One gemm_big configuration launched `iters` times (for rocprofv3 --pmc passes):
python scripts/gemm_big_one.py M N K epi variant iters"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from mxserve import ops
    M, N, K, epi, variant, iters = (int(a) for a in sys.argv[1:7])
    dev = torch.device("cuda:0")
    x = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
    w = ((torch.rand(N, K, device=dev) * 2 - 1) * K ** -0.5).to(torch.bfloat16)
    y = torch.empty(M, N // 2 if epi else N, device=dev, dtype=torch.bfloat16)
    for _ in range(iters):
        assert ops.ext().gemm_big(y, x, w, epi, variant)
    torch.cuda.synchronize()
    print("ok", M, N, K, epi, variant, iters)


if __name__ == "__main__":
    main()
