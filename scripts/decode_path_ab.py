#!/usr/bin/env python3
"""Pure-decode steps above 256 rows (Llama-3.2-1B, ctx 4000): the prefill chain (llama.py _forward_pf,
gemm_pf / prefill-bucket tables) against the decode chain (_forward_fused, the decode table's tuned
forms), each a captured hipGraph of the whole forward + lm_head, timed over replays.  Also the
decode chain's non-attention time (the same graph with attention skipped is not separable, so
attention kernels are timed alone and subtracted).  JSON lines per batch."""
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    Bs = [int(x) for x in (sys.argv[1].split(",") if len(sys.argv) > 1 else "256,320,384,448".split(","))]
    from mxserve.models.config import get_model_config
    from mxserve.models.llama import AttnMetadata, build_model
    from mxserve.ops import decode_gemm, prefill_pf
    dev = torch.device("cuda:0")
    cfg = get_model_config("meta-llama/Llama-3.2-1B-Instruct")
    m = build_model(cfg, dev)
    m.init_random()
    m.prepare_fused_prefill(tuning=True, max_rows=6144 + 448)
    w = m.w
    norm = ("add_norm",) if m.fuse_residual else None
    shapes = {"qkv": (w["l0.qkv"], 0, ("rope", m.nh, m.nkv, m.hd)), "o": (w["l0.o"], 0, norm),
              "gate_up": (w["l0.gate_up"], 1), "down": (w["l0.down"], 0, norm), "lm_head": (m.lm_head_weight(), 0)}
    with torch.inference_mode():
        decode_gemm.tune(shapes, Bs, dev)
        prefill_pf.tune({k: (v[0], v[1]) for k, v in shapes.items() if k != "lm_head"}, 6144 + 448, dev)
        fw = {"o": (w["l0.o"], None, prefill_pf.CODE_RESID), "down": (w["l0.down"], None, prefill_pf.CODE_RESID)}
        prefill_pf.tune_fused(fw, 6144 + 448, dev)
    ctx = 4000
    for B in Bs:
        nbps = math.ceil((ctx + 1) / 16)
        kv = torch.randn(B * nbps + 16, cfg.num_layers, 2, m.nkv, 16, cfg.head_dim, dtype=torch.bfloat16,
                         device=dev) * 0.1
        i32 = dict(dtype=torch.int32, device=dev)
        bt = torch.randperm(B * nbps, device=dev).view(B, nbps).to(torch.int32)
        md = AttnMetadata(positions=torch.full((B,), ctx, dtype=torch.int64, device=dev),
                          slot_mapping=bt[:, -1].long() * 16 + (ctx % 16), block_tables=bt,
                          seq_lens=torch.full((B,), ctx + 1, **i32), query_start_loc=torch.arange(B + 1, **i32),
                          logits_indices=torch.arange(B, device=dev), num_decodes=B, num_prefills=0,
                          num_prefill_tokens=0, max_query_len=1, max_seq_len=8192)
        ids = torch.randint(0, cfg.vocab_size, (B,), device=dev)
        res = {"B": B}
        for path, pf in (("prefill_chain", True), ("decode_chain", False)):
            m.pf_decode = pf
            with torch.inference_mode():
                s = torch.cuda.Stream()
                s.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(s):
                    for _ in range(2):
                        m.compute_logits(m.forward(ids, md, kv))
                torch.cuda.current_stream().wait_stream(s)
                torch.cuda.synchronize()
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    m.compute_logits(m.forward(ids, md, kv))
            for _ in range(3):
                g.replay()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ts = []
            for _ in range(5):
                e0.record()
                for _ in range(10):
                    g.replay()
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1) / 10)
            ts.sort()
            res[path + "_ms"] = round(ts[2], 4)
            del g
        print(json.dumps(res), flush=True)
        del kv
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
