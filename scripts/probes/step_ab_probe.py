#!/usr/bin/env python3
"""Step-level A/B of engine settings that can change in-process: one mixed engine step of the headline
workload (B decode rows at ~CTX context + one CHUNK-token prefill after PREFIX cached tokens;
Llama-3.2-1B forward + logits, the engine's own routing tables loaded by building an LLMEngine with
the bench's limits), each mode timed in turn, rounds interleaved.  Modes (STEP_MODES, comma list):
base, hblt_off (mxserve/ops/prefill_hblt.py table off), var0 (prefill attention forced to the
default v3 variant instead of the split / paired choice), no_overlap (prefill-chunk attention on the
main stream), no_overlap_var0.  MS_CASES="B:CTX:CHUNK:PREFIX,..."; one JSON line per case."""
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    from mxserve.config import EngineArgs
    from mxserve.engine.engine import LLMEngine
    from mxserve.models.llama import AttnMetadata
    from mxserve import ops
    from mxserve.models import llama
    from mxserve.ops import prefill_hblt
    all_modes = {"base": {}, "hblt_off": {"hblt": "off"}, "var0": {"pv": 0x100}, "no_overlap": {"ov": False},
                 "no_overlap_var0": {"ov": False, "pv": 0x100}}
    names = [m for m in os.environ.get("STEP_MODES", "base,hblt_off").split(",") if m]
    pv0, ov0, hb0 = ops._PREFILL_VERSION, llama._ATTN_OVERLAP, prefill_hblt.MODE

    def apply(mode):
        st = all_modes[mode]
        ops._PREFILL_VERSION = st.get("pv", pv0)
        llama._ATTN_OVERLAP = st.get("ov", ov0)
        prefill_hblt.MODE = st.get("hblt", hb0)
    dev = torch.device("cuda:0")
    eng = LLMEngine(EngineArgs(model="meta-llama/Llama-3.2-1B-Instruct", device="cuda", max_num_seqs=448,
                               cuda_graph_max_bs=448, max_num_batched_tokens=6144, max_model_len=8192,
                               num_gpu_blocks=4096))
    m, cfg = eng.runner.model, eng.runner.cfg
    i32 = dict(dtype=torch.int32, device=dev)
    # "B:CTX:CHUNK:PREFIX[+CHUNK:PREFIX...]": B decode rows, then one or more prefill sequences
    cases = []
    for c in os.environ.get("MS_CASES", "300:4250:2400:1600,300:4250:4000:0,400:4250:1200:2800,"
                                        "350:4250:5700:0,0:0:4000:0").split(","):
        head, *more = c.split("+")
        B, ctx, chunk, prefix = (int(x) for x in head.split(":"))
        cases.append((B, ctx, [(chunk, prefix)] + [tuple(int(x) for x in m.split(":")) for m in more]))
    for B, ctx, pf in cases:
        torch.manual_seed(0)
        dl = torch.randint(max(1, ctx - 250), ctx + 250, (B,)).tolist() if B else []
        lens = [d + 1 for d in dl] + [p + c for c, p in pf]
        nbs = [math.ceil(n / 16) for n in lens]
        nb = sum(nbs) + 8
        kv = torch.randn(nb, cfg.num_layers, 2, m.nkv, 16, cfg.head_dim, dtype=torch.bfloat16, device=dev) * 0.1
        perm = torch.randperm(nb - 8, device=dev).to(torch.int32)
        bt = torch.zeros(B + len(pf), max(nbs), **i32)
        o = 0
        for i, n in enumerate(nbs):
            bt[i, :n] = perm[o:o + n]
            o += n
        chunk = sum(c for c, _ in pf)
        pos_d = torch.tensor(dl, dtype=torch.int64, device=dev)
        pos_p = torch.cat([torch.arange(p, p + c, dtype=torch.int64, device=dev) for c, p in pf])
        positions = torch.cat([pos_d, pos_p])
        rows = torch.cat([torch.arange(B, device=dev)] + [torch.full((c,), B + j, device=dev) for j, (c, _) in enumerate(pf)])
        slot = bt[rows, (positions // 16)].long() * 16 + positions % 16
        cum = [0]
        for c, _ in pf:
            cum.append(cum[-1] + c)
        qsl = torch.tensor(list(range(B + 1)) + [B + x for x in cum[1:]], **i32)
        md = AttnMetadata(positions=positions, slot_mapping=slot, block_tables=bt,
                          seq_lens=torch.tensor(lens, **i32), query_start_loc=qsl,
                          logits_indices=torch.cat([torch.arange(B, device=dev),
                                                    torch.tensor([B + x - 1 for x in cum[1:]], device=dev)]),
                          num_decodes=B, num_prefills=len(pf), num_prefill_tokens=chunk,
                          max_query_len=max(c for c, _ in pf), max_seq_len=max(lens),
                          prefill_query_start_loc=torch.tensor(cum, **i32),
                          sample_seq=torch.arange(B + len(pf), **i32))
        ids = torch.randint(0, cfg.vocab_size, (B + chunk,), device=dev)
        times = {k: [] for k in names}
        outs = {}
        with torch.inference_mode():
            for _ in range(8):
                for mode in times:
                    apply(mode)
                    for _ in range(2):
                        outs[mode] = m.compute_logits(m.forward(ids, md, kv))
                    torch.cuda.synchronize()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(5):
                        m.compute_logits(m.forward(ids, md, kv))
                    e1.record()
                    torch.cuda.synchronize()
                    times[mode].append(e0.elapsed_time(e1) / 5)
        apply("base")
        r = {k: round(sorted(v)[len(v) // 2], 3) for k, v in times.items()}
        b = names[0]
        diff = {k: round((outs[k].float() - outs[b].float()).abs().max().item(), 4) for k in names[1:]}
        print(json.dumps({"B": B, "ctx": ctx, "prefills": pf, "rows": B + chunk, "ms": r,
                          "time_vs_" + b: {k: round(r[k] / r[b], 4) for k in names[1:]},
                          "logits_max_abs_diff": diff,
                          "all_ms": {k: [round(x, 3) for x in v] for k, v in times.items()}}), flush=True)
        del kv


if __name__ == "__main__":
    main()
