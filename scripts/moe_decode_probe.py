#!/usr/bin/env python3
"""Mixtral-8x7B expert layer at decode batches: the LDS-tiled grouped GEMM (moe_gemm.hip) vs the
grouped form of the decode GEMM kernel (gemm_decode.hip), every configuration, timed inside
hipGraphs.  JSON lines: gemm, tokens T, config, microseconds, GB/s over the weights of the experts
that received rows.  Each T ends with the whole layer on both paths and their max difference."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def route(T, E, k, dev, g):
    logits = torch.randn(T, E, device=dev, generator=g)
    w, ids = torch.topk(torch.softmax(logits, -1), k, dim=-1)
    return (w / w.sum(-1, keepdim=True)).float(), ids.to(torch.int32)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", default="4,16,32,64,128,256")
    ap.add_argument("--hidden", type=int, default=4096)
    ap.add_argument("--inter", type=int, default=14336)
    ap.add_argument("--experts", type=int, default=8)
    ap.add_argument("--top", type=int, default=6, help="configurations printed per (gemm, T)")
    a = ap.parse_args()
    from mxserve.ops import decode_gemm as dg
    from mxserve.ops import ext, moe
    dev = torch.device("cuda:0")
    moe.DECODE = False
    g = torch.Generator(device=dev).manual_seed(0)
    E, H, I, k = a.experts, a.hidden, a.inter, 2
    w13 = (torch.randn(E, 2 * I, H, device=dev, generator=g) * 0.02).to(torch.bfloat16)
    w2 = (torch.randn(E, H, I, device=dev, generator=g) * 0.02).to(torch.bfloat16)
    for T in [int(t) for t in a.tokens.split(",")]:
        x = (torch.randn(T, H, device=dev, generator=g)).to(torch.bfloat16)
        tw, ids = route(T, E, k, dev, g)
        offs = torch.empty(E + 1, dtype=torch.int32, device=dev)
        perm = torch.full((T * k,), -1, dtype=torch.int32, device=dev)
        inv = torch.empty(T * k, dtype=torch.int32, device=dev)
        ext().moe_align(offs, perm, ids, 0, E, inv)
        active = int((offs[1:] > offs[:-1]).sum().item())
        xs = x.index_select(0, (perm.clamp(min=0).long() // k))
        R = T * k
        h = torch.empty(R, I, dtype=torch.bfloat16, device=dev)
        ys = torch.empty(R, H, dtype=torch.bfloat16, device=dev)
        part = torch.empty(8 * R * max(2 * I, H), dtype=torch.float32, device=dev)
        ref = moe.fused_experts(x, w13, w2, tw, ids)
        t_old = dg._graph_time(lambda: moe.fused_experts(x, w13, w2, tw, ids))
        print(json.dumps({"gemm": "layer_grouped_lds", "T": T, "active_experts": active, "us": round(t_old, 1),
                          "GBps_w": round(active * 3 * I * H * 2 / t_old / 1e3, 1)}), flush=True)
        for name, (w, epi, N, K, o) in {"w13": (w13, 1, 2 * I, H, h), "w2": (w2, 0, H, I, ys)}.items():
            xin = xs if name == "w13" else h
            res = []
            for cfg in dg.candidates(min(T, 256), N, K, epi, all_mf=True, mt=False):
                sk = cfg[3]
                if cfg[2] > 2:
                    continue
                pp = part[: sk * R * N].view(sk, R, N) if sk > 1 else None
                if not moe._mdg(o, xin, w, offs, pp, T, cfg, epi):
                    continue
                us = dg._graph_time(lambda: moe._mdg(o, xin, w, offs, pp, T, cfg, epi))
                res.append((cfg, us))
            res.sort(key=lambda r: r[1])
            for c, us in res[: a.top]:
                print(json.dumps({"gemm": name, "T": T, "cfg": c, "us": round(us, 1),
                                  "GBps_w": round(active * N * K * 2 / us / 1e3, 1)}), flush=True)
        moe.DECODE = True
        new = moe.fused_experts(x, w13, w2, tw, ids)
        t_new = dg._graph_time(lambda: moe.fused_experts(x, w13, w2, tw, ids))
        moe.DECODE = False
        err = (new.float() - ref.float()).abs().max().item()
        print(json.dumps({"gemm": "layer_decode_kernel", "T": T, "active_experts": active, "us": round(t_new, 1),
                          "GBps_w": round(active * 3 * I * H * 2 / t_new / 1e3, 1), "max_abs_err_vs_grouped": err,
                          "ref_max": ref.float().abs().max().item()}), flush=True)


if __name__ == "__main__":
    main()
