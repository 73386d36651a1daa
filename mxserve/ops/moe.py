"""MoE expert computation on the GPU (K15-K17), Mixtral 8x7B top-2, experts sharded over EP ranks.

fused_experts: the moe_align counting sort buckets the (token, slot) assignments by local expert,
the rows are gathered once, and two MFMA grouped-GEMM launches (csrc/kernels/moe_gemm.hip) run
every local expert over exactly its rows -- gate_up with SiLU*mul fused into the epilogue, then
down -- before the combine kernel gathers each token's top-k rows back (weighted, fp32 accumulate,
one bf16 write per element; csrc/kernels/moe.hip).  No host sync anywhere, so decode steps
stay hipGraph-capturable and prefill costs two launches instead of 2 x E_local GEMMs.
_fused_experts_loop keeps the per-expert formulation (dense over all tokens at small T, sorted rows
otherwise) for shapes the grouped kernel does not tile.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

DENSE_MAX_TOKENS = 256
# grouped kernel up to this many tokens (decode / mixed steps, graph-capturable); above it the
# per-expert hipBLASLt GEMMs over sorted rows are faster (profiles/r1_moe_layer_mixtral.jsonl:
# grouped 0.82 / 0.86 ms vs 0.89 / 1.22 ms at T = 64 / 256; 2.77 vs 2.01 ms at T = 2048)
GROUPED_MAX_TOKENS = 512


def _silu_mul(h: torch.Tensor) -> torch.Tensor:
    from . import silu_mul
    return silu_mul(h)


def combine_weights(topk_w: torch.Tensor, topk_ids: torch.Tensor, e_local: int, offset: int) -> torch.Tensor:
    """[T, E_local] fp32 routing weights (sum over the top-k slots that picked each local expert)."""
    T, K = topk_ids.shape
    local = topk_ids.long() - offset
    valid = (local >= 0) & (local < e_local)
    cw = torch.zeros(T, e_local, dtype=torch.float32, device=topk_w.device)
    cw.scatter_add_(1, local.clamp(0, e_local - 1), torch.where(valid, topk_w.float(), torch.zeros_like(topk_w)))
    return cw


def _fused_experts_loop(x, w13, w2, topk_w, topk_ids, expert_offset):
    """Reference-structured fallback (shapes the grouped kernel does not tile): dense per-expert
    GEMMs for small T, per-expert GEMMs over moe_align-sorted rows otherwise."""
    T, H = x.shape
    e_local = w13.shape[0]
    if T <= DENSE_MAX_TOKENS:
        cw = combine_weights(topk_w, topk_ids, e_local, expert_offset)
        out = torch.zeros(T, H, dtype=torch.float32, device=x.device)
        for e in range(e_local):
            y = F.linear(_silu_mul(F.linear(x, w13[e])), w2[e])
            out.add_(y.float() * cw[:, e:e + 1])
        return out.to(x.dtype)
    from . import ext
    K = topk_ids.shape[1]
    ids = topk_ids.to(torch.int32).contiguous()
    offs = torch.empty(e_local + 1, dtype=torch.int32, device=x.device)
    perm = torch.empty(T * K, dtype=torch.int32, device=x.device)
    ext().moe_align(offs, perm, ids, expert_offset, e_local)
    o = offs.tolist()
    rows = perm[:o[-1]].long()
    tok = rows // K
    xs = x.index_select(0, tok)
    ys = torch.empty(o[-1], H, dtype=x.dtype, device=x.device)
    for e in range(e_local):
        a, b = o[e], o[e + 1]
        if b > a:
            ys[a:b] = F.linear(_silu_mul(F.linear(xs[a:b], w13[e])), w2[e])
    wts = topk_w.reshape(-1).index_select(0, rows).unsqueeze(1)
    out = torch.zeros(T, H, dtype=torch.float32, device=x.device)
    out.index_add_(0, tok, ys.float() * wts)
    return out.to(x.dtype)


def fused_experts(x: torch.Tensor, w13: torch.Tensor, w2: torch.Tensor, topk_w: torch.Tensor,
                  topk_ids: torch.Tensor, expert_offset: int = 0) -> torch.Tensor:
    """K15 align -> gather -> K16 grouped GEMM (gate_up with SiLU*mul fused in its epilogue) ->
    K16 grouped GEMM (down) -> K17 weighted scatter-add.  Entirely on the device (no host sync):
    graph-capturable for decode.  Large prefill chunks take the per-expert hipBLASLt loop."""
    from . import ext
    T, H = x.shape
    if T > GROUPED_MAX_TOKENS:
        return _fused_experts_loop(x, w13, w2, topk_w, topk_ids, expert_offset)
    K = topk_ids.shape[1]
    e_local, two_i, _ = w13.shape
    dev = x.device
    ids = topk_ids.to(torch.int32).contiguous()
    offs = torch.empty(e_local + 1, dtype=torch.int32, device=dev)
    perm = torch.full((T * K,), -1, dtype=torch.int32, device=dev)
    inv = torch.empty(T * K, dtype=torch.int32, device=dev)
    ext().moe_align(offs, perm, ids, expert_offset, e_local, inv)
    rows = perm.clamp(min=0).long()
    tok = rows // K
    xs = x.index_select(0, tok)  # rows past the routed count are ignored by the GEMMs
    h = torch.empty(T * K, two_i // 2, dtype=x.dtype, device=dev)
    ys = torch.empty(T * K, H, dtype=x.dtype, device=dev)
    # split-K for the down projection when the routed rows leave too few workgroups to stream the
    # weights (decode; one expert per rank under EP): aim at ~1024 workgroups
    tiles = min(e_local, T * K) + -(-T * K // 128)
    split = max(1, min(8, (two_i // 2) // 64, -(-1024 // ((H // 128) * tiles))))
    part = torch.empty(split, T * K, H, dtype=torch.float32, device=dev) if split > 1 else None
    # gate_up likewise (fp32 slices over [gate; up], SiLU*mul applied when they are summed) when its
    # grid is small too: one local expert per rank
    split13 = max(1, min(4, H // 64, -(-1024 // ((two_i // 128) * tiles))))
    if split13 > 1:
        part13 = torch.empty(split13, T * K, two_i, dtype=torch.float32, device=dev)
        ok13 = ext().moe_grouped_gemm(ys.new_empty(0, two_i), xs, w13.contiguous(), offs, False, split13, part13)
        if ok13:
            ext().silu_mul_partials(h, part13)
    else:
        ok13 = ext().moe_grouped_gemm(h, xs, w13.contiguous(), offs, True)
    if not (ok13 and ext().moe_grouped_gemm(ys, h, w2.contiguous(), offs, False, split, part)):
        return _fused_experts_loop(x, w13, w2, topk_w, topk_ids, expert_offset)
    out = torch.empty(T, H, dtype=x.dtype, device=dev)
    if part is not None:
        ext().moe_combine_partials(out, part, topk_w.float().contiguous(), inv)  # K17 over the K slices
    else:
        ext().moe_combine(out, ys, topk_w.float().contiguous(), inv)  # K17
    return out
