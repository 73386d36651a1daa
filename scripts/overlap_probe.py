#!/usr/bin/env python3
"""Does a bandwidth-bound decode step overlap a compute-bound prefill chunk on one MI355X?

Kernel level: one layer's paged decode attention (B=256, ctx 4000: ~2.1 GB of KV, HBM-bound) on one
HIP stream against a prefill-sized GEMM (hipBLASLt, M=8192, MFMA-bound) on another.
Model level: Llama-3.2-1B decode steps (B=256, ctx 4000) on stream D while an 8192-token prefill
chunk runs on stream P, vs the two back to back (what a mixed engine step does today).
Prints JSON lines: serial vs concurrent wall, per stream priority setting."""
from __future__ import annotations

import json
import math
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def ev():
    return torch.cuda.Event(enable_timing=True)


def timed(fn, iters=10, warmup=2) -> float:
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    s, e = ev(), ev()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def concurrent(fa, na: int, fb, nb: int, sa, sb) -> tuple:
    """na calls of fa on stream sa and nb of fb on sb, started together; (wall, a_end, b_end) ms."""
    torch.cuda.synchronize()
    start = ev()
    ea, eb = ev(), ev()
    start.record()
    sa.wait_event(start)
    sb.wait_event(start)
    with torch.cuda.stream(sa):
        for _ in range(na):
            fa()
        ea.record()
    with torch.cuda.stream(sb):
        for _ in range(nb):
            fb()
        eb.record()
    torch.cuda.synchronize()
    ta, tb = start.elapsed_time(ea), start.elapsed_time(eb)
    return max(ta, tb), ta, tb


def main():
    from mxserve import ops
    from mxserve.models.config import get_model_config
    from mxserve.models.llama import AttnMetadata, build_model
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    out = []
    B, ctx = 256, 4000
    cfg = get_model_config("meta-llama/Llama-3.2-1B-Instruct")
    nbps = math.ceil((ctx + 1) / 16)
    # ---------------- kernel level
    nkv, D, nh = cfg.num_kv_heads, cfg.head_dim, cfg.num_heads
    nb1 = B * nbps + 16
    kv1 = torch.randn(nb1, 2, nkv, 16, D, dtype=torch.bfloat16, device=dev) * 0.1
    bt1 = torch.randperm(nb1 - 16, device=dev)[:B * nbps].view(B, nbps).to(torch.int32)
    sl1 = torch.full((B,), ctx + 1, dtype=torch.int32, device=dev)
    q1 = torch.randn(B, nh, D, dtype=torch.bfloat16, device=dev)
    attn = lambda: ops.paged_attention_decode(q1, kv1, bt1, sl1, 0.125, 8192)  # noqa: E731
    x = torch.randn(8192, 2048, dtype=torch.bfloat16, device=dev)
    wgu = torch.randn(16384, 2048, dtype=torch.bfloat16, device=dev) * 0.02
    a8 = torch.randn(8192, 8192, dtype=torch.bfloat16, device=dev)
    wd = torch.randn(2048, 8192, dtype=torch.bfloat16, device=dev) * 0.02
    gemms = {"gate_up_8192": lambda: torch.nn.functional.linear(x, wgu),
             "down_8192": lambda: torch.nn.functional.linear(a8, wd)}
    t_attn = timed(attn, 20)
    out.append({"op": "decode_attn_layer", "ms": round(t_attn, 4)})
    for prio in (0, -1):
        sd = torch.cuda.Stream(priority=prio)  # decode stream (priority -1 = high)
        sp = torch.cuda.Stream(priority=0)
        for name, g in gemms.items():
            t_g = timed(g, 20)
            n_a = max(1, round(4 * t_g / t_attn))
            serial = 4 * t_g + n_a * t_attn
            wall, ta, tb = concurrent(attn, n_a, g, 4, sd, sp)
            wall2, _, _ = concurrent(attn, n_a, g, 4, sd, sp)
            out.append({"op": "kernel_overlap", "gemm": name, "gemm_ms": round(t_g, 4), "attn_calls": n_a,
                        "gemm_calls": 4, "decode_prio": prio, "serial_ms": round(serial, 3),
                        "concurrent_ms": round(min(wall, wall2), 3), "attn_stream_ms": round(ta, 3),
                        "gemm_stream_ms": round(tb, 3), "speedup": round(serial / min(wall, wall2), 3)})
            print(json.dumps(out[-1]), flush=True)
    del kv1, a8, wd, wgu, x
    torch.cuda.empty_cache()

    # ---------------- model level
    m = build_model(cfg, dev)
    m.init_random()
    T, P = 8192, 2
    per = T // P
    nbp = per // 16
    nb = B * nbps + P * nbp + 32
    kv = torch.randn(nb, cfg.num_layers, 2, m.nkv, 16, D, dtype=torch.bfloat16, device=dev) * 0.1
    bt = torch.randperm(B * nbps, device=dev).view(B, nbps).to(torch.int32)
    sl = torch.full((B,), ctx + 1, dtype=torch.int32, device=dev)
    i32 = dict(dtype=torch.int32, device=dev)
    pos = torch.full((B,), ctx, dtype=torch.int64, device=dev)
    md_d = AttnMetadata(positions=pos, slot_mapping=bt[:, -1].long() * 16 + (ctx % 16), block_tables=bt, seq_lens=sl,
                        query_start_loc=torch.arange(B + 1, **i32), logits_indices=torch.arange(B, device=dev),
                        num_decodes=B, num_prefills=0, num_prefill_tokens=0, max_query_len=1, max_seq_len=8192)
    ids_d = torch.randint(0, cfg.vocab_size, (B,), device=dev)
    base = B * nbps
    btp = (base + torch.arange(P * nbp, device=dev)).view(P, nbp).to(torch.int32)
    posp = torch.arange(per, device=dev).repeat(P)
    slotp = (btp.long().repeat_interleave(16, dim=1) * 16 + torch.arange(16, device=dev).repeat(nbp)).view(-1)
    qsl = torch.arange(0, T + 1, per, **i32)
    md_p = AttnMetadata(positions=posp, slot_mapping=slotp, block_tables=btp, seq_lens=torch.full((P,), per, **i32),
                        query_start_loc=qsl, logits_indices=(qsl[1:] - 1).long(), num_decodes=0, num_prefills=P,
                        num_prefill_tokens=T, max_query_len=per, max_seq_len=per, prefill_query_start_loc=qsl,
                        sample_seq=torch.arange(P, **i32))
    ids_p = torch.randint(0, cfg.vocab_size, (T,), device=dev)

    def dec():
        with torch.inference_mode():
            m.compute_logits(m.forward(ids_d, md_d, kv))

    def pre():
        with torch.inference_mode():
            m.compute_logits(m.forward(ids_p, md_p, kv))
    t_d, t_p = timed(dec, 10), timed(pre, 5)
    out.append({"op": "model_alone", "decode_step_ms": round(t_d, 3), "prefill_chunk_ms": round(t_p, 3)})
    print(json.dumps(out[-1]), flush=True)
    for prio in (0, -1):
        sd = torch.cuda.Stream(priority=prio)
        sp = torch.cuda.Stream(priority=0)
        n_d = max(1, round(t_p / t_d))
        res = []
        for _ in range(3):
            res.append(concurrent(dec, n_d, pre, 1, sd, sp))
        wall, ta, tb = min(res)
        serial = t_p + n_d * t_d
        out.append({"op": "model_overlap", "decode_prio": prio, "decode_steps": n_d, "serial_ms": round(serial, 3),
                    "concurrent_ms": round(wall, 3), "decode_stream_ms": round(ta, 3), "prefill_stream_ms": round(tb, 3),
                    "decode_step_ms_under_prefill": round(ta / n_d, 3), "speedup": round(serial / wall, 3)})
        print(json.dumps(out[-1]), flush=True)
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/overlap_probe.jsonl", "w") as f:
        for r in out:
            f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
