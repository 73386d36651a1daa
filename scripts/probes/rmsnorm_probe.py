#!/usr/bin/env python3
"""RMSNorm (plain and with the residual add) at Llama-3.2-1B's hidden size over decode and prefill
row counts; JSON lines with us and TB/s (bytes read + written).  MXS_RMS_BLOCK=1 selects the
workgroup-per-row kernel, unset the wave-per-row one (csrc/kernels/norm_act.hip)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    from mxserve import ops
    dev = torch.device("cuda:0")
    H = int(os.environ.get("RMS_H", "2048"))
    for rows in (1, 64, 320, 2048, 4096, 6144, 8192):
        x = torch.randn(rows, H, device=dev, dtype=torch.bfloat16)
        r = torch.randn(rows, H, device=dev, dtype=torch.bfloat16)
        w = torch.ones(H, device=dev, dtype=torch.bfloat16)
        for name, fn, nbytes in (("plain", lambda: ops.rms_norm(x, w, 1e-5), 2 * rows * H * 2),
                                 ("add", lambda: ops.fused_add_rms_norm(x, r, w, 1e-5), 4 * rows * H * 2)):
            for _ in range(5):
                fn()
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for _ in range(50):
                    fn()
            ts = []
            for _ in range(5):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                g.replay()
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1) * 1e3 / 50)
            us = sorted(ts)[2]
            print(json.dumps({"form": "block" if os.environ.get("MXS_RMS_BLOCK") == "1" else "wave", "op": name,
                              "rows": rows, "H": H, "us": round(us, 2), "TBps": round(nbytes / us / 1e6, 2)}), flush=True)


if __name__ == "__main__":
    main()
