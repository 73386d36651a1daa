#!/usr/bin/env python3
"""Re-measure the Llama-3.2-1B decode-GEMM choices (each projection priced with its epilogue, as
the engine's capture-time tuner does) at the given batch buckets, ignoring the stored table
(MXS_RETUNE=1 semantics); with MXS_TUNED_SAVE=1 / MXS_TUNED_DIR the results land in a table file
that can be merged into mxserve/ops/tuned/.  Prints one JSON line per (projection, bucket)."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--buckets", default="1,2,4,8,16,24,32,48,64")
    a = ap.parse_args()
    os.environ["MXS_RETUNE"] = "1"
    from mxserve.models.config import get_model_config
    from mxserve.models.llama import build_model
    from mxserve.ops import decode_gemm
    dev = torch.device("cuda:0")
    m = build_model(get_model_config("meta-llama/Llama-3.2-1B-Instruct"), dev)
    m.init_random()
    w = m.w
    norm = ("add_norm",) if m.fuse_residual else None
    decode_gemm.tune({"qkv": (w["l0.qkv"], 0, ("rope", m.nh, m.nkv, m.hd)), "o": (w["l0.o"], 0, norm),
                      "gate_up": (w["l0.gate_up"], 1), "down": (w["l0.down"], 0, norm),
                      "lm_head": (m.lm_head_weight(), 0)}, [int(b) for b in a.buckets.split(",")], dev)
    for r in decode_gemm.TABLE.report:
        print(json.dumps({k: r.get(k) for k in ("proj", "M", "chosen", "cfg", "us", "hipblaslt_us", "source")}),
              flush=True)


if __name__ == "__main__":
    main()
