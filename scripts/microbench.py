#!/usr/bin/env python3
"""Component timings on one MI355X: decode step (graph), prefill chunk, attention kernels alone,
and the projection GEMMs, for Llama-3.2-1B at the bench shape (ISL 4000).  Prints JSON lines."""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters=20, warmup=3):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def timeit_graph(fn, iters=20):
    """Kernel time without host launch gaps: `iters` calls captured in one hipGraph."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.inference_mode(), torch.cuda.graph(g):
        for _ in range(iters):
            fn()
    g.replay()
    torch.cuda.synchronize()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    g.replay()
    en.record()
    torch.cuda.synchronize()
    return st.elapsed_time(en) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="meta-llama/Llama-3.2-1B-Instruct")
    ap.add_argument("--ctx", type=int, default=4000)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--prefill", type=int, default=8192)
    a = ap.parse_args()
    from mxserve import ops
    from mxserve.models.config import get_model_config
    from mxserve.models.llama import AttnMetadata, build_model
    dev = torch.device("cuda:0")
    cfg = get_model_config(a.model)
    m = build_model(cfg, dev)
    m.init_random()
    B, ctx = a.batch, a.ctx
    nbps = math.ceil((ctx + 1) / 16)
    nb = B * nbps + 16
    kv = torch.randn(nb, cfg.num_layers, 2, m.nkv, 16, cfg.head_dim, dtype=torch.bfloat16, device=dev) * 0.1
    bt = torch.randperm(nb - 16, device=dev)[:B * nbps].view(B, nbps).to(torch.int32)
    sl = torch.full((B,), ctx + 1, dtype=torch.int32, device=dev)
    out = []

    # ---- decode attention kernel alone (one layer)
    q = torch.randn(B, m.nh, cfg.head_dim, dtype=torch.bfloat16, device=dev)
    t = timeit(lambda: ops.paged_attention_decode(q, kv[:, 0], bt, sl, 0.125, ctx + 1))
    byts = B * (ctx + 1) * m.nkv * cfg.head_dim * 2 * 2
    out.append({"op": "paged_decode_attn_layer", "B": B, "ctx": ctx, "ms": t, "GBps": byts / t / 1e6})
    t8k = timeit(lambda: ops.paged_attention_decode(q, kv[:, 0], bt, sl, 0.125, 8192))
    out.append({"op": "paged_decode_attn_layer_graphgrid8192", "ms": t8k, "GBps": byts / t8k / 1e6})
    # fp8 (e4m3fn) cache of the same shape: half the bytes per token
    kv8 = torch.empty(nb, 2, m.nkv, 16, cfg.head_dim, dtype=torch.uint8, device=dev)
    kv8.copy_((kv[:, 0].float() * 16).to(torch.float8_e4m3fn).view(torch.uint8))
    t = timeit(lambda: ops.paged_attention_decode(q, kv8, bt, sl, 0.125, ctx + 1, k_scale=1 / 16, v_scale=1 / 16))
    out.append({"op": "paged_decode_attn_layer_fp8kv", "B": B, "ctx": ctx, "ms": t, "GBps": byts / 2 / t / 1e6})

    # ---- full decode step (eager and graph)
    pos = torch.full((B,), ctx, dtype=torch.int64, device=dev)
    slots = (bt[:, -1].long() * 16 + (ctx % 16))
    ids = torch.randint(0, cfg.vocab_size, (B,), device=dev)
    md = AttnMetadata(positions=pos, slot_mapping=slots, block_tables=bt, seq_lens=sl,
                      query_start_loc=torch.arange(B + 1, dtype=torch.int32, device=dev),
                      logits_indices=torch.arange(B, device=dev), num_decodes=B, num_prefills=0,
                      num_prefill_tokens=0, max_query_len=1, max_seq_len=8192)
    temp = torch.ones(B, device=dev)

    def step():
        h = m.forward(ids, md, kv)
        lg = m.compute_logits(h)
        return ops.sample(lg, temp, torch.ones(B, device=dev), torch.zeros(B, dtype=torch.int32, device=dev),
                          torch.arange(B, device=dev), torch.zeros(B, dtype=torch.int64, device=dev))

    # decode projection GEMMs: the graph-time tuner picks the MFMA kernel or hipBLASLt per projection
    from mxserve.ops import decode_gemm
    wd = m.w
    with torch.inference_mode():
        rows = decode_gemm.tune({"qkv": (wd["l0.qkv"], 0), "o": (wd["l0.o"], 0), "gate_up": (wd["l0.gate_up"], 1),
                                 "down": (wd["l0.down"], 0), "lm_head": (m.lm_head_weight(), 0)}, [B], dev)
    for r in rows:
        out.append(dict(r, op="decode_gemm_tune"))
    mode = decode_gemm.MODE
    decode_gemm.MODE = "off"
    with torch.inference_mode():
        g0 = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            step()
        torch.cuda.current_stream().wait_stream(s)
        with torch.cuda.graph(g0):
            step()
        tg0 = timeit(g0.replay, iters=20)
    decode_gemm.MODE = mode
    out.append({"op": "decode_step_hipblaslt_only", "B": B, "ctx": ctx, "graph_ms": tg0})
    del g0
    with torch.inference_mode():
        te = timeit(step, iters=10)
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            step()
        torch.cuda.current_stream().wait_stream(s)
        with torch.cuda.graph(g):
            step()
        tg = timeit(g.replay, iters=20)
    out.append({"op": "decode_step", "B": B, "ctx": ctx, "eager_ms": te, "graph_ms": tg,
                "tok_per_s": B / tg * 1e3})
    # same decode step over an fp8 (e4m3fn) copy of the cache (--kv-cache-dtype fp8)
    kv8 = torch.empty(kv.shape, dtype=torch.uint8, device=dev)
    for li in range(cfg.num_layers):
        kv8[:, li].copy_((kv[:, li].float() * 16).to(torch.float8_e4m3fn).view(torch.uint8))
    scales_bf16 = m.kv_scales
    m.kv_scales = [{"k_scale": 1 / 16, "v_scale": 1 / 16} for _ in range(cfg.num_layers)]

    def step8():
        h = m.forward(ids, md, kv8)
        lg = m.compute_logits(h)
        return ops.sample(lg, temp, torch.ones(B, device=dev), torch.zeros(B, dtype=torch.int32, device=dev),
                          torch.arange(B, device=dev), torch.zeros(B, dtype=torch.int64, device=dev))

    with torch.inference_mode():
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            step8()
        torch.cuda.current_stream().wait_stream(s)
        g8 = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g8):
            step8()
        tg8 = timeit(g8.replay, iters=20)
    out.append({"op": "decode_step_fp8kv", "B": B, "ctx": ctx, "graph_ms": tg8, "tok_per_s": B / tg8 * 1e3})
    m.kv_scales = scales_bf16
    del kv8, g8

    # ---- prefill chunk (ctx 0, T tokens as 2 sequences)
    T = a.prefill
    nseq = 2
    per = T // nseq
    pb = math.ceil(per / 16)
    bt2 = torch.arange(nseq * pb, device=dev, dtype=torch.int32).view(nseq, pb)
    pos2 = torch.cat([torch.arange(per) for _ in range(nseq)]).to(dev)
    slots2 = torch.cat([bt2[i].long().repeat_interleave(16)[:per] * 16 + torch.arange(per, device=dev) % 16
                        for i in range(nseq)])
    qsl = torch.tensor([i * per for i in range(nseq + 1)], dtype=torch.int32, device=dev)
    md2 = AttnMetadata(positions=pos2, slot_mapping=slots2, block_tables=bt2,
                       seq_lens=torch.full((nseq,), per, dtype=torch.int32, device=dev), query_start_loc=qsl,
                       logits_indices=qsl[1:].long() - 1, num_decodes=0, num_prefills=nseq,
                       num_prefill_tokens=T, max_query_len=per, max_seq_len=per, prefill_query_start_loc=qsl)
    ids2 = torch.randint(0, cfg.vocab_size, (T,), device=dev)
    with torch.inference_mode():
        tp = timeit(lambda: m.compute_logits(m.forward(ids2, md2, kv)), iters=5)
    flops = 2 * T * (cfg.num_params() - cfg.vocab_size * cfg.hidden_size)
    out.append({"op": "prefill_chunk", "T": T, "ms": tp, "TFLOPs_linear": flops / tp / 1e9})
    qp = torch.randn(T, m.nh, cfg.head_dim, dtype=torch.bfloat16, device=dev)
    ta = timeit(lambda: ops.paged_attention_prefill(qp, kv[:, 0], bt2, qsl, md2.seq_lens, 0.125, per))
    af = 4 * nseq * per * per / 2 * cfg.head_dim * m.nh
    out.append({"op": "prefill_attn_layer", "T": T, "ms": ta, "TFLOPs": af / ta / 1e9})

    # ---- GEMMs (prefill M=T and decode M=B)
    H, I = cfg.hidden_size, cfg.intermediate_size
    shapes = {"qkv": ((m.nh + 2 * m.nkv) * cfg.head_dim, H), "o": (H, m.nh * cfg.head_dim), "gate_up": (2 * I, H),
              "down": (H, I), "lm_head": (cfg.vocab_size, H)}
    for Mrows in (T, B, 64, 16, 1) if B not in (64, 16, 1) else (T, B):
        for name, (N, K) in shapes.items():
            if name == "lm_head" and Mrows == T:
                continue
            x = torch.randn(Mrows, K, dtype=torch.bfloat16, device=dev)
            w = torch.randn(N, K, dtype=torch.bfloat16, device=dev)
            impls = {"hipblaslt": lambda: F.linear(x, w)}
            if Mrows <= 256:
                impls["decode_gemm_tuned"] = lambda: ops.linear(x, w)
            for impl, fn in impls.items():
                tt = timeit_graph(fn)
                out.append({"op": f"gemm_{name}", "impl": impl, "M": Mrows, "N": N, "K": K, "ms": tt,
                            "TFLOPs": 2 * Mrows * N * K / tt / 1e9, "GBps_w": N * K * 2 / tt / 1e6})
    # elementwise
    x = torch.randn(T, H, dtype=torch.bfloat16, device=dev)
    w = torch.ones(H, dtype=torch.bfloat16, device=dev)
    r = torch.randn_like(x)
    tt = timeit(lambda: ops.fused_add_rms_norm(x, r, w, 1e-5))
    out.append({"op": "fused_add_rmsnorm", "T": T, "ms": tt, "GBps": 4 * T * H * 2 / tt / 1e6})
    gu = torch.randn(T, 2 * I, dtype=torch.bfloat16, device=dev)
    tt = timeit(lambda: ops.silu_mul(gu))
    out.append({"op": "silu_mul", "T": T, "ms": tt, "GBps": 3 * T * I * 2 / tt / 1e6})
    for o in out:
        print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in o.items()}), flush=True)


if __name__ == "__main__":
    main()
