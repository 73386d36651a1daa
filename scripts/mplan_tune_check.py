#!/usr/bin/env python3
"""Start-up M-plan tuning on a model the packaged table does not cover (Llama-3-8B, random init):
tuning time, how many buckets got a plan, and ops.linear vs F.linear at a few row counts."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from mxserve import ops
    from mxserve.config import EngineArgs
    from mxserve.engine.engine import LLMEngine
    t0 = time.time()
    eng = LLMEngine(EngineArgs(model="meta-llama/Meta-Llama-3-8B-Instruct", device="cuda", num_gpu_blocks=4096,
                               max_model_len=8192, max_num_seqs=64, load_format="random"))
    rep = getattr(eng.runner, "mplan_report", None)
    dev = torch.device("cuda:0")
    tab = ops._MPLAN.get(dev, {})
    print(json.dumps({"engine_build_s": round(time.time() - t0, 1), "mplan_report": rep,
                      "buckets_with_plan": {k: len(v) for k, v in tab.items()}}), flush=True)
    w = eng.runner.model.w
    from mxserve.ops import mplan
    for name in ("l0.qkv", "l0.o", "l0.gate_up", "l0.down"):
        W = w[name]
        for M in (1300, 4200, 4350, 6200, 8192):
            x = torch.randn(M, W.shape[1], device=dev, dtype=W.dtype)
            a = mplan._time_us(lambda: torch.nn.functional.linear(x, W), 10)
            b = mplan._time_us(lambda: ops.linear(x, W), 10)
            print(json.dumps({"w": name, "M": M, "plan": ops._mplan(M, W.shape[0], W.shape[1], dev),
                              "linear_us": round(a, 1), "ops_linear_us": round(b, 1)}), flush=True)


if __name__ == "__main__":
    main()
