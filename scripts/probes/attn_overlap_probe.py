#!/usr/bin/env python3
"""Mixed-step attention: the decode rows' attention (HBM-bound) and the prefill chunk's attention
(MFMA / VALU-bound) of one layer, back to back on one stream vs the prefill on a second stream.
Llama-3.2-1B heads (32 q / 8 kv, D 64); B decode sequences of ~CTX tokens, one prefill chunk of
CHUNK new tokens after PREFIX cached ones (the headline's mixed steps: ~300 decode rows + ~2.4k
prefill tokens).  OV_CASES="B:CTX:CHUNK:PREFIX,..." overrides; one JSON line per case and mode."""
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    from mxserve import ops
    dev = torch.device("cuda:0")
    hq, hkv, D = 32, 8, 64
    cases = [tuple(int(x) for x in c.split(":")) for c in
             os.environ.get("OV_CASES", "300:4250:2400:1600,300:4250:4000:0,400:4250:1200:2800").split(",")]
    for B, ctx, chunk, prefix in cases:
        torch.manual_seed(0)
        dl = torch.randint(ctx - 250, ctx + 250, (B,), dtype=torch.int32)
        lens = dl.tolist() + [prefix + chunk]
        nbs = [-(-n // 16) for n in lens]
        nb = sum(nbs)
        kv = (torch.randn(nb, 2, hkv, 16, D, device=dev) * 0.5).to(torch.bfloat16)
        perm = torch.randperm(nb, device=dev).to(torch.int32)
        bt = torch.zeros(len(lens), max(nbs), dtype=torch.int32, device=dev)
        o = 0
        for i, n in enumerate(nbs):
            bt[i, :n] = perm[o:o + n]
            o += n
        qd = torch.randn(B, hq, D, device=dev, dtype=torch.bfloat16)
        qp = torch.randn(chunk, hq, D, device=dev, dtype=torch.bfloat16)
        sl_d = dl.to(dev)
        sl_p = torch.tensor([prefix + chunk], dtype=torch.int32, device=dev)
        qsl = torch.tensor([0, chunk], dtype=torch.int32, device=dev)
        bt_d, bt_p = bt[:B], bt[B:]
        od, op = torch.empty_like(qd), torch.empty_like(qp)
        side = torch.cuda.Stream(device=dev)
        side_hi = torch.cuda.Stream(device=dev, priority=-1)
        main_s = torch.cuda.current_stream(dev)
        scale = D ** -0.5

        def dec():
            ops.paged_attention_decode(qd, kv, bt_d, sl_d, scale, int(dl.max()), out=od)

        def pre():
            ops.paged_attention_prefill(qp, kv, bt_p, qsl, sl_p, scale, chunk, out=op)

        def seq_mode():
            dec()
            pre()

        def ov_pre_first():
            side.wait_stream(main_s)
            with torch.cuda.stream(side):
                pre()
            dec()
            main_s.wait_stream(side)

        def ov_dec_first():
            side.wait_stream(main_s)
            dec()
            with torch.cuda.stream(side):
                pre()
            main_s.wait_stream(side)

        def ov_hiprio():
            side_hi.wait_stream(main_s)
            with torch.cuda.stream(side_hi):
                pre()
            dec()
            main_s.wait_stream(side_hi)

        modes = {"decode_only": dec, "prefill_only": pre, "sequential": seq_mode,
                 "overlap_prefill_first": ov_pre_first, "overlap_decode_first": ov_dec_first,
                 "overlap_prefill_hiprio": ov_hiprio}
        times = {k: [] for k in modes}
        ref_d, ref_p = None, None
        for rnd in range(5):
            for name, fn in modes.items():
                for _ in range(3):
                    fn()
                torch.cuda.synchronize()
                if name == "sequential" and rnd == 0:
                    ref_d, ref_p = od.clone(), op.clone()
                if name.startswith("overlap") and rnd == 0:
                    assert torch.equal(od, ref_d) and torch.equal(op, ref_p), name
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(16):  # one step's 16 layers
                    fn()
                e1.record()
                torch.cuda.synchronize()
                times[name].append(e0.elapsed_time(e1) / 16 * 1000)
        res = {k: round(sorted(v)[2], 1) for k, v in times.items()}
        kv_bytes = sum(dl.tolist()) * hkv * D * 2 * 2
        print(json.dumps({"B": B, "ctx": ctx, "chunk": chunk, "prefix": prefix, "us_per_layer": res,
                          "decode_TBps": round(kv_bytes / res["decode_only"] / 1e6, 2),
                          "overlap_gain": round(res["sequential"] / min(res["overlap_prefill_first"],
                                                                         res["overlap_decode_first"]), 3)}),
              flush=True)
        del kv


if __name__ == "__main__":
    main()
