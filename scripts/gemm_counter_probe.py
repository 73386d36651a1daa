#!/usr/bin/env python3
"""Runs a few launches of one prefill GEMM variant for a rocprofv3 --pmc pass:
python scripts/gemm_counter_probe.py <kernel: v7|pf|lib> <M> <N> <K> [epi]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from mxserve import ops
    kern, M, N, K = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
    epi = int(sys.argv[5]) if len(sys.argv) > 5 else 0
    dev = torch.device("cuda:0")
    x = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
    w = ((torch.rand(N, K, device=dev) * 2 - 1) * K ** -0.5).to(torch.bfloat16)
    y = torch.empty(M, N // 2 if epi else N, device=dev, dtype=torch.bfloat16)
    for _ in range(5):
        if kern == "v7":
            ops.ext().gemm_big(y, x, w, epi, 7)
        elif kern == "pf":
            ops.gemm_pf(x, w, epi, y, 16)
        else:
            torch.nn.functional.linear(x, w)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
