"""MoE expert computation on the GPU (K15-K17).

Two regimes (Mixtral 8x7B, top-2, experts sharded over EP ranks):
  * decode / small T (<= DENSE_MAX_TOKENS): the step is bound by streaming the local experts'
    weights, and with >= ~32 tokens every expert is hit anyway, so each local expert runs over all
    tokens and the results are combined with a [T, E_local] routing-weight matrix (zero for
    unrouted pairs).  No host sync, so the step stays hipGraph-capturable.
  * prefill / large T: tokens are bucketed by expert with the moe_align counting-sort kernel and
    each expert runs a GEMM over only its rows (no wasted FLOPs); the weighted results are
    scatter-added back to token order.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

DENSE_MAX_TOKENS = 256


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


def fused_experts(x: torch.Tensor, w13: torch.Tensor, w2: torch.Tensor, topk_w: torch.Tensor,
                  topk_ids: torch.Tensor, expert_offset: int = 0) -> torch.Tensor:
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
