#!/usr/bin/env python3
"""Kernel-level breakdown of the two step kinds of the headline workload (Llama-3.2-1B, ISL 4000):
an 8192-token prefill chunk (two 4096-token prompts) and a B=256 decode step at ctx 4000, each run
`--iters` times eagerly so `rocprofv3 --kernel-trace --stats -- python scripts/step_profile.py`
attributes GPU time per kernel.  --which prefill|decode|both."""
from __future__ import annotations

import argparse
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--which", default="both")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--chunk", type=int, default=8192)
    ap.add_argument("--tuned", action="store_true",
                    help="load the decode GEMM choices the engine would use (packaged table / tuner)")
    a = ap.parse_args()
    from mxserve.models.config import get_model_config
    from mxserve.models.llama import AttnMetadata, build_model
    dev = torch.device("cuda:0")
    cfg = get_model_config("meta-llama/Llama-3.2-1B-Instruct")
    m = build_model(cfg, dev)
    m.init_random()
    B, ctx, T = a.batch, 4000, a.chunk
    P = max(1, T // 4096)
    per = T // P
    nbps, nbp = math.ceil((ctx + 1) / 16), per // 16
    nb = B * nbps + P * nbp + 32
    kv = torch.randn(nb, cfg.num_layers, 2, m.nkv, 16, cfg.head_dim, dtype=torch.bfloat16, device=dev) * 0.1
    i32 = dict(dtype=torch.int32, device=dev)
    bt = torch.randperm(B * nbps, device=dev).view(B, nbps).to(torch.int32)
    md_d = AttnMetadata(positions=torch.full((B,), ctx, dtype=torch.int64, device=dev),
                        slot_mapping=bt[:, -1].long() * 16 + (ctx % 16), block_tables=bt,
                        seq_lens=torch.full((B,), ctx + 1, **i32), query_start_loc=torch.arange(B + 1, **i32),
                        logits_indices=torch.arange(B, device=dev), num_decodes=B, num_prefills=0,
                        num_prefill_tokens=0, max_query_len=1, max_seq_len=8192)
    btp = (B * nbps + torch.arange(P * nbp, device=dev)).view(P, nbp).to(torch.int32)
    qsl = torch.arange(0, T + 1, per, **i32)
    md_p = AttnMetadata(positions=torch.arange(per, device=dev).repeat(P),
                        slot_mapping=(btp.long().repeat_interleave(16, dim=1) * 16
                                      + torch.arange(16, device=dev).repeat(nbp)).view(-1),
                        block_tables=btp, seq_lens=torch.full((P,), per, **i32), query_start_loc=qsl,
                        logits_indices=(qsl[1:] - 1).long(), num_decodes=0, num_prefills=P, num_prefill_tokens=T,
                        max_query_len=per, max_seq_len=per, prefill_query_start_loc=qsl, sample_seq=torch.arange(P, **i32))
    if a.tuned:  # the engine's decode GEMM / fused-epilogue choices for this batch bucket
        from mxserve.ops import decode_gemm
        w = m.w
        norm = ("add_norm",) if m.fuse_residual else None
        decode_gemm.tune({"qkv": (w["l0.qkv"], 0, ("rope", m.nh, m.nkv, m.hd)), "o": (w["l0.o"], 0, norm),
                          "gate_up": (w["l0.gate_up"], 1), "down": (w["l0.down"], 0, norm),
                          "lm_head": (m.lm_head_weight(), 0)}, [B], dev)
        print({r["proj"]: r["cfg"] for r in decode_gemm.TABLE.report})
        for r in decode_gemm.TABLE.report:  # per projection: the pick and both timings
            print({k: r.get(k) for k in ("M", "proj", "chosen", "cfg", "us", "hipblaslt_us", "source")})
    ids_d = torch.randint(0, cfg.vocab_size, (B,), device=dev)
    ids_p = torch.randint(0, cfg.vocab_size, (T,), device=dev)
    with torch.inference_mode():
        for _ in range(a.iters):
            if a.which in ("both", "prefill"):
                m.compute_logits(m.forward(ids_p, md_p, kv))
            if a.which in ("both", "decode"):
                m.compute_logits(m.forward(ids_d, md_d, kv))
    torch.cuda.synchronize()
    print("done")


if __name__ == "__main__":
    main()
