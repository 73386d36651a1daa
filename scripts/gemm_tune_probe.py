#!/usr/bin/env python3
"""Prefill GEMM probe: hipBLASLt default heuristic vs PyTorch TunableOp (benchmarks every
hipBLASLt / rocBLAS solution for the exact shape) on the Llama-3.2-1B / Llama-3-8B prefill
projections.  Prints one JSON line per (model, T, projection, mode)."""
from __future__ import annotations

import json
import os
import sys

import torch

SHAPES = {  # name: (K, N) of y[T, N] = x[T, K] . w[N, K]^T
    "1b": {"qkv": (2048, 3072), "o": (2048, 2048), "gate_up": (2048, 16384), "down": (8192, 2048)},
    "1b_lm": {"lm_head": (2048, 128256)},
    "8b": {"qkv": (4096, 6144), "o": (4096, 4096), "gate_up": (4096, 28672), "down": (14336, 4096)},
}


def bench(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e-3


def main():
    models = sys.argv[1].split(",") if len(sys.argv) > 1 else ["1b"]
    Ts = [int(t) for t in (sys.argv[2].split(",") if len(sys.argv) > 2 else ["2048", "4096", "8192"])]
    dev = torch.device("cuda")
    tun = torch.cuda.tunable
    out_file = os.environ.get("MXS_TUNE_FILE", "gpurun_out/tunableop_results.csv")
    for mode in ("default", "tunableop"):
        if mode == "tunableop":
            tun.enable(True)
            tun.tuning_enable(True)
            tun.set_filename(out_file)
            tun.set_max_tuning_duration(60)
        for m in models:
            for T in Ts:
                for name, (K, N) in SHAPES[m].items():
                    x = torch.randn(T, K, device=dev, dtype=torch.bfloat16)
                    w = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02
                    if mode == "tunableop":
                        torch.nn.functional.linear(x, w)  # tunes this shape
                        torch.cuda.synchronize()
                    s = bench(lambda: torch.nn.functional.linear(x, w))
                    print(json.dumps({"model": m, "T": T, "proj": name, "mode": mode, "us": round(s * 1e6, 1),
                                      "tflops": round(2 * T * K * N / s / 1e12, 1)}), flush=True)
    if tun.is_enabled():
        tun.write_file_on_exit(True)


if __name__ == "__main__":
    main()
