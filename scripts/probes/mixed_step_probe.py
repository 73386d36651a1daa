#!/usr/bin/env python3
"""One mixed engine step of the headline workload (Llama-3.2-1B forward + logits): B decode rows at
~CTX tokens of context plus one prefill chunk of CHUNK tokens after PREFIX cached ones, timed with
events, with the mixed-step attention overlap off and on (mxserve/models/llama.py _ATTN_OVERLAP)
alternately in one process.  MS_CASES="B:CTX:CHUNK:PREFIX,..."; one JSON line per case."""
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    from mxserve.models import llama
    from mxserve.models.config import get_model_config
    from mxserve.models.llama import AttnMetadata, build_model
    dev = torch.device("cuda:0")
    cfg = get_model_config("meta-llama/Llama-3.2-1B-Instruct")
    m = build_model(cfg, dev)
    m.init_random()
    i32 = dict(dtype=torch.int32, device=dev)
    cases = [tuple(int(x) for x in c.split(":")) for c in
             os.environ.get("MS_CASES", "300:4250:2400:1600,300:4250:4000:0,400:4250:1200:2800").split(",")]
    for B, ctx, chunk, prefix in cases:
        torch.manual_seed(0)
        dl = torch.randint(ctx - 250, ctx + 250, (B,)).tolist()  # context before this step's token
        plen = prefix + chunk
        lens = [d + 1 for d in dl] + [plen]
        nbs = [math.ceil(n / 16) for n in lens]
        nb = sum(nbs) + 8
        kv = torch.randn(nb, cfg.num_layers, 2, m.nkv, 16, cfg.head_dim, dtype=torch.bfloat16, device=dev) * 0.1
        perm = torch.randperm(nb - 8, device=dev).to(torch.int32)
        bt = torch.zeros(B + 1, max(nbs), **i32)
        o = 0
        for i, n in enumerate(nbs):
            bt[i, :n] = perm[o:o + n]
            o += n
        pos_d = torch.tensor(dl, dtype=torch.int64, device=dev)
        pos_p = torch.arange(prefix, plen, dtype=torch.int64, device=dev)
        positions = torch.cat([pos_d, pos_p])
        rows = torch.cat([torch.arange(B, device=dev), torch.full((chunk,), B, device=dev)])
        slot = bt[rows, (positions // 16)].long() * 16 + positions % 16
        qsl = torch.tensor(list(range(B + 1)) + [B + chunk], **i32)
        md = AttnMetadata(positions=positions, slot_mapping=slot, block_tables=bt,
                          seq_lens=torch.tensor(lens, **i32), query_start_loc=qsl,
                          logits_indices=torch.cat([torch.arange(B, device=dev), torch.tensor([B + chunk - 1], device=dev)]),
                          num_decodes=B, num_prefills=1, num_prefill_tokens=chunk, max_query_len=chunk,
                          max_seq_len=max(lens), prefill_query_start_loc=torch.tensor([0, chunk], **i32),
                          sample_seq=torch.arange(B + 1, **i32))
        ids = torch.randint(0, cfg.vocab_size, (B + chunk,), device=dev)
        # the same step as two independent forwards: the decode rows, the prefill chunk
        md_d = AttnMetadata(positions=pos_d, slot_mapping=slot[:B], block_tables=bt[:B],
                            seq_lens=torch.tensor(lens[:B], **i32), query_start_loc=torch.arange(B + 1, **i32),
                            logits_indices=torch.arange(B, device=dev), num_decodes=B, num_prefills=0,
                            num_prefill_tokens=0, max_query_len=1, max_seq_len=max(lens[:B]),
                            sample_seq=torch.arange(B, **i32))
        md_p = AttnMetadata(positions=pos_p, slot_mapping=slot[B:], block_tables=bt[B:],
                            seq_lens=torch.tensor([plen], **i32), query_start_loc=torch.tensor([0, chunk], **i32),
                            logits_indices=torch.tensor([chunk - 1], device=dev), num_decodes=0, num_prefills=1,
                            num_prefill_tokens=chunk, max_query_len=chunk, max_seq_len=plen,
                            prefill_query_start_loc=torch.tensor([0, chunk], **i32),
                            sample_seq=torch.zeros(1, **i32))
        main_s, side = torch.cuda.current_stream(dev), torch.cuda.Stream(device=dev)

        def combined():
            return m.compute_logits(m.forward(ids, md, kv))

        def split_seq():
            a = m.compute_logits(m.forward(ids[:B], md_d, kv))
            b = m.compute_logits(m.forward(ids[B:], md_p, kv))
            return torch.cat([a, b])

        def split_par():
            side.wait_stream(main_s)
            with torch.cuda.stream(side):
                b = m.compute_logits(m.forward(ids[B:], md_p, kv))
            a = m.compute_logits(m.forward(ids[:B], md_d, kv))
            main_s.wait_stream(side)
            return torch.cat([a, b])

        # the decode rows' forward replayed from a hipGraph (as the engine's decode steps run)
        g = None
        if os.environ.get("MS_GRAPH", "1") == "1":
            with torch.inference_mode():
                for _ in range(2):
                    m.compute_logits(m.forward(ids[:B], md_d, kv))
                torch.cuda.synchronize()
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    glog = m.compute_logits(m.forward(ids[:B], md_d, kv))

        def split_seq_graph():
            g.replay()
            b = m.compute_logits(m.forward(ids[B:], md_p, kv))
            return torch.cat([glog, b])

        def split_par_graph():
            side.wait_stream(main_s)
            with torch.cuda.stream(side):
                b = m.compute_logits(m.forward(ids[B:], md_p, kv))
            g.replay()
            main_s.wait_stream(side)
            return torch.cat([glog, b])

        def split_par_graph_rev():  # decode graph on the side stream, prefill on the main one
            side.wait_stream(main_s)
            with torch.cuda.stream(side):
                g.replay()
            b = m.compute_logits(m.forward(ids[B:], md_p, kv))
            main_s.wait_stream(side)
            return torch.cat([glog, b])

        modes = {"combined": (combined, 0), "combined_attn_overlap": (combined, 1), "split_sequential": (split_seq, 0),
                 "split_parallel": (split_par, 0)}
        if g is not None:
            modes.update({"split_seq_graph": (split_seq_graph, 0), "split_par_graph": (split_par_graph, 0),
                          "split_par_graph_rev": (split_par_graph_rev, 0)})
        if os.environ.get("MS_MODES"):  # e.g. "combined_attn_overlap" under rocprofv3
            modes = {k: v for k, v in modes.items() if k in os.environ["MS_MODES"].split(",")}
        times = {k: [] for k in modes}
        outs = {}
        with torch.inference_mode():
            for rnd in range(6):
                for name, (fn, ov) in modes.items():
                    llama._ATTN_OVERLAP = bool(ov)
                    for _ in range(2):
                        outs[name] = fn()
                    torch.cuda.synchronize()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(5):
                        fn()
                    e1.record()
                    torch.cuda.synchronize()
                    times[name].append(e0.elapsed_time(e1) / 5)
        r = {k: round(sorted(v)[len(v) // 2], 3) for k, v in times.items()}
        base = outs.get("combined", next(iter(outs.values())))
        diff = {k: round((outs[k].float() - base.float()).abs().max().item(), 4) for k in outs}
        print(json.dumps({"B": B, "ctx": ctx, "chunk": chunk, "prefix": prefix, "ms": r,
                          "gain_vs_combined": {k: round(r.get("combined", v) / v, 3) for k, v in r.items()},
                          "logits_max_diff": diff}), flush=True)
        del kv


if __name__ == "__main__":
    main()
