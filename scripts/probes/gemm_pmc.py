#!/usr/bin/env python3
"""One prefill GEMM launched `iters` times for `rocprofv3 --pmc` passes: argv kernel (w4 | pf) M N K
epi [iters].  Random [-1, 1) operands."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    from mxserve import ops
    kern = sys.argv[1]
    M, N, K, epi = (int(a) for a in sys.argv[2:6])
    iters = int(sys.argv[6]) if len(sys.argv) > 6 else 10
    dev = torch.device("cuda:0")
    x = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
    w = ((torch.rand(N, K, device=dev) * 2 - 1) * K ** -0.5).to(torch.bfloat16)
    r = (torch.rand(M, N, device=dev) * 2 - 1).to(torch.bfloat16) if epi == 2 else None
    y = torch.empty(M, N // 2 if epi == 1 else N, device=dev, dtype=torch.bfloat16)
    for _ in range(iters):
        if kern == "w4":
            assert ops.gemm_w4(x, w, epi, y, resid=r) is not None
        else:
            assert ops.gemm_pf(x, w, epi, y, 16, resid=r) is not None
    torch.cuda.synchronize()
    print("done", kern, M, N, K, epi)


if __name__ == "__main__":
    main()
