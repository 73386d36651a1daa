"""Per-layer decode microbench of a tensor-parallel shard (BASELINE config 4,
Llama-3-70B at TP = 8 over xGMI): the four projection GEMMs of ONE rank's shard, chosen by the
decode-GEMM tuner (mxserve/ops/decode_gemm.py) with cold weights, and the two fused all-reduce +
residual-add + RMSNorm epilogues (custom_allreduce.hip car_add_rmsnorm_kernel) across the TP group,
against the weight-streaming floor (shard bytes / HBM bandwidth).

Usable two ways, both one process per rank with `torch.distributed` initialised (comm.init_distributed):
  * real node (one GPU per rank): the whole layer chain -- qkv, o + AR/add/norm, gate_up + SiLU,
    down + AR/add/norm -- captured in one hipGraph and replayed on every rank together;
  * ranks sharing one GPU ("virtual ranks", what a 1-GPU box can run): the GEMM chain is timed on
    rank 0 alone while the others wait (it is per rank and identical on every rank), the fused
    epilogues with every rank running them concurrently, and the layer is their sum.
Attention is left out (its cost scales with context, not with the shard); the report says so.

  torchrun --nproc-per-node 8 -m mxserve.tools.tp_layer_bench --buckets 1,8,32,64,128
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

HBM_TBPS = 6.0  # achievable HBM read bandwidth of one MI355X (cdna guides: ~6.0-6.3 TB/s measured)

LLAMA3_70B = dict(hidden=8192, heads=64, kv_heads=8, head_dim=128, inter=28672)


def shard_shapes(tp: int, m=LLAMA3_70B) -> dict:
    """{name: (N, K, epi)} of one rank's projections at TP = tp (column-parallel qkv / gate_up,
    row-parallel o / down)."""
    H, hd = m["hidden"], m["head_dim"]
    q = m["heads"] // tp * hd
    kv = max(1, m["kv_heads"] // tp) * hd
    i = m["inter"] // tp
    return {"qkv": (q + 2 * kv, H, 0), "o": (H, q, 0), "gate_up": (2 * i, H, 1), "down": (H, i, 0)}


def _graph_us(fn, iters: int = 20, sync=None) -> float:
    """Microseconds per call of fn, 20 calls captured in one hipGraph.  sync (the group's barrier):
    collectives inside fn -- every rank starts each replay together, so a rank's clock does not
    include waiting for a peer that is still capturing."""
    sync = sync or (lambda: None)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(iters):
            fn()
    sync()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    sync()
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


def run(buckets=(1, 8, 32, 64, 128), shared: bool = False, barrier=None, log=print) -> dict:
    """Returns the report on rank 0 (others: {}).  `barrier()` is the group's CPU barrier."""
    import torch.distributed as dist
    from .. import ops
    from ..ops import decode_gemm
    from ..parallel.comm import get_tp, tp_linear_add_rms_norm
    st = get_tp()
    tp, rank = st.tp_size, st.tp_rank
    dev = torch.device("cuda", torch.cuda.current_device())
    barrier = barrier or (lambda: dist.barrier(group=st.cpu_group))
    shapes = shard_shapes(tp)
    g = torch.Generator(device="cpu").manual_seed(1234 + rank)
    ws = {k: (torch.randn(N, K, generator=g) * K ** -0.5).to(torch.bfloat16).to(dev) for k, (N, K, _) in shapes.items()}
    H = LLAMA3_70B["hidden"]
    norm_w = torch.ones(H, dtype=torch.bfloat16, device=dev)
    bytes_layer = sum(N * K * 2 for N, K, _ in shapes.values())
    floor_us = bytes_layer / (HBM_TBPS * 1e12) * 1e6
    # the decode-GEMM table for these shard shapes (persisted per device like every tuned table)
    t0 = time.time()
    # each projection priced with its epilogue, as the engine's capture-time tuning does: qkv with the
    # rope / cache write, o / down with the residual add + norm (slab-consuming forms win there)
    hq, hkv = LLAMA3_70B["heads"] // tp, max(1, LLAMA3_70B["kv_heads"] // tp)
    specs = {"qkv": ("rope", hq, hkv, LLAMA3_70B["head_dim"]), "o": ("add_norm",), "gate_up": None,
             "down": ("add_norm",)}
    tshapes = {k: (ws[k], shapes[k][2]) + ((specs[k],) if specs[k] else ()) for k in shapes}
    if rank == 0 or not shared:
        decode_gemm.tune(tshapes, list(buckets), dev)
    barrier()
    if shared and rank != 0:  # same table on every rank (the fused epilogue's split-K choice)
        decode_gemm.tune(tshapes, list(buckets), dev)
    tune_s = time.time() - t0
    rows = []
    car = st.custom_ar
    for M in buckets:
        h = (torch.randn(M, H, generator=g) * 0.5).to(torch.bfloat16).to(dev)
        residual = torch.randn(M, H, generator=g).to(torch.bfloat16).to(dev)
        attn = (torch.randn(M, shapes["o"][1], generator=g) * 0.5).to(torch.bfloat16).to(dev)
        copies = {k: decode_gemm.weight_copies(w, cap=8) for k, w in ws.items()}  # cold weights
        it = [0]

        def w_(k):
            c = copies[k]
            return c[it[0] % len(c)]

        def gemms():  # one rank's projections of the layer, weights cold; partials not reduced
            it[0] += 1
            ops.linear(h, w_("qkv"))
            ops.linear(attn, w_("o"))
            a = ops.gate_up_silu(h, w_("gate_up"))
            ops.linear(a, w_("down"))

        def layer():  # the TP chain: GEMMs + the two fused all-reduce / add / norm epilogues
            it[0] += 1
            ops.linear(h, w_("qkv"))
            h1, _ = tp_linear_add_rms_norm(attn, w_("o"), residual, norm_w, 1e-5)
            a = ops.gate_up_silu(h1, w_("gate_up"))
            tp_linear_add_rms_norm(a, w_("down"), residual, norm_w, 1e-5)

        row = {"M": M}
        per = {}
        if rank == 0:
            for k in shapes:
                x = {"qkv": h, "o": attn, "gate_up": h, "down": None}[k]
                if k == "down":
                    x = (torch.randn(M, shapes["down"][1], generator=g) * 0.5).to(torch.bfloat16).to(dev)
                fn = (lambda x=x, k=k: ops.gate_up_silu(x, w_(k))) if k == "gate_up" else \
                    (lambda x=x, k=k: ops.linear(x, w_(k)))
                us = _graph_us(lambda fn=fn: (it.__setitem__(0, it[0] + 1), fn()))
                N, K, _ = shapes[k]
                cfg = decode_gemm.TABLE.lookup(M, N, K, shapes[k][2])
                per[k] = {"us": round(us, 2), "TBps": round(N * K * 2 / us / 1e6, 2),
                          "kernel": "hipblaslt" if cfg is None else str(list(cfg))}
            row["gemms"] = per
        barrier()
        if car is not None and car.can_add_rms_norm(residual):
            x_bf = (torch.randn(M, H, generator=g) * 0.1).to(torch.bfloat16).to(dev)
            barrier()
            t_ar = _graph_us(lambda: car.add_rms_norm(residual, norm_w, 1e-5, x=x_bf), sync=barrier)
            barrier()

            def unfused():
                y = car.all_reduce(x_bf, out=torch.empty_like(x_bf))
                ops.fused_add_rms_norm(y, residual, norm_w, 1e-5)
            t_un = _graph_us(unfused, sync=barrier)
            barrier()
            row["ar_add_norm_us"] = round(t_ar, 2)
            row["ar_then_add_norm_us"] = round(t_un, 2)
        if shared:
            if rank == 0:
                t_g = _graph_us(gemms)
                row["gemm_chain_us"] = round(t_g, 2)
                row["layer_us"] = round(t_g + 2 * row.get("ar_add_norm_us", 0.0), 2)
                row["layer_method"] = "GEMM chain on rank 0 alone + 2 x fused epilogue timed with all ranks"
            barrier()
        else:
            barrier()
            row["layer_us"] = round(_graph_us(layer, sync=barrier), 2)
            row["layer_method"] = "whole chain captured and replayed on every rank together"
            barrier()
        if rank == 0:
            row["floor_us"] = round(floor_us, 2)
            row["vs_floor"] = round(row["layer_us"] / floor_us, 3) if "layer_us" in row else None
            rows.append(row)
            log(json.dumps(row))
        del copies
        torch.cuda.empty_cache()
    if rank != 0:
        return {}
    return {"model": "Llama-3-70B", "tp": tp, "shared_gpu": shared, "hbm_tbps_floor": HBM_TBPS,
            "shard_weight_bytes_per_layer": bytes_layer, "shapes": {k: list(v) for k, v in shapes.items()},
            "attention": "excluded (context-dependent, not sharded weight traffic)", "tune_s": round(tune_s, 1),
            "rows": rows}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--buckets", default="1,8,32,64,128")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    from ..parallel.comm import init_distributed
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = torch.cuda.device_count()
    shared = ndev < world
    torch.cuda.set_device(local % ndev)
    dev = torch.device("cuda", local % ndev)
    # ranks sharing a GPU: control over gloo, all-reduces through the IPC mesh (custom all-reduce)
    init_distributed(world, backend="gloo" if shared else "nccl", device=dev, timeout_s=300)
    res = run(tuple(int(b) for b in a.buckets.split(",")), shared=shared)
    if res:
        print("TPLAYER " + json.dumps(res), flush=True)
        if a.out:
            with open(a.out, "w") as f:
                json.dump(res, f, indent=1)
    import torch.distributed as dist
    dist.barrier()
    dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
