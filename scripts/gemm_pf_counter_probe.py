#!/usr/bin/env python3
"""One gemm_pf shape launched `iters` times for `rocprofv3 --pmc` passes (counters per dispatch):
argv: M N K epi min_iters [iters].  Random [-1, 1) operands (cdna_hip_programming.md §5.4 rule 25)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from mxserve import ops
    M, N, K, epi, mi = (int(a) for a in sys.argv[1:6])
    iters = int(sys.argv[6]) if len(sys.argv) > 6 else 10
    dev = torch.device("cuda:0")
    x = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
    w = ((torch.rand(N, K, device=dev) * 2 - 1) * K ** -0.5).to(torch.bfloat16)
    y = torch.empty(M, N // 2 if epi == 1 else N, device=dev, dtype=torch.bfloat16)
    for _ in range(iters):
        assert ops.gemm_pf(x, w, epi, y, mi) is not None
    torch.cuda.synchronize()
    print("done", M, N, K, epi, mi)


if __name__ == "__main__":
    main()
