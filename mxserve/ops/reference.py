"""Plain-PyTorch reference implementations of every engine op.

These run the CPU backend (BASELINE config 1) and are the fp32 oracles the HIP-kernel tests
compare against.  Layout contracts shared with `csrc/kernels/*.hip`:

* paged KV cache of one layer: a view `[num_blocks, 2, Hkv, BS, D]` (block stride may be larger:
  the engine allocates one block-major tensor `[NB, L, 2, Hkv, BS, D]` so a block holds all layers'
  K and V contiguously - SURVEY.md §5.8 "block-major layout" for P->D transfer).
  K is stored token-major `[BS][D]`; V is stored dim-major `[D][BS]` (so both the QK^T and the
  P·V MFMA operands are 16-byte vector loads from global memory).
* `slot_mapping[t] = block_id * BS + offset`, `-1` = skip (padding).
* cos/sin cache: `[max_pos, D]` fp32, first D/2 columns cos, last D/2 sin (rotate-half RoPE).
"""
from __future__ import annotations

import math
from typing import Optional

import torch
import torch.nn.functional as F


def rms_norm(x: torch.Tensor, w: torch.Tensor, eps: float) -> torch.Tensor:
    xf = x.float()
    y = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)
    return (y * w.float()).to(x.dtype)


def fused_add_rms_norm(x: torch.Tensor, residual: torch.Tensor, w: torch.Tensor, eps: float):
    """r = x + residual; y = rmsnorm(r) * w.  Returns (y, r).  r is rounded to x.dtype first
    (matches the kernel: the residual stream is stored in the activation dtype)."""
    r = (x.float() + residual.float()).to(x.dtype)
    return rms_norm(r, w, eps), r


def silu_mul(gu: torch.Tensor) -> torch.Tensor:
    d = gu.shape[-1] // 2
    g, u = gu[..., :d].float(), gu[..., d:].float()
    return (F.silu(g) * u).to(gu.dtype)


def build_cos_sin_cache(head_dim: int, max_pos: int, theta: float,
                        rope_scaling: Optional[dict] = None, device="cpu") -> torch.Tensor:
    inv_freq = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=torch.float64) / head_dim))
    if rope_scaling is not None:  # llama3 frequency-dependent scaling
        factor = rope_scaling["factor"]
        lf, hf = rope_scaling["low_freq_factor"], rope_scaling["high_freq_factor"]
        old = rope_scaling["original_max_position_embeddings"]
        low_wl, high_wl = old / lf, old / hf
        wl = 2 * math.pi / inv_freq
        smooth = (old / wl - lf) / (hf - lf)
        scaled = torch.where(wl > low_wl, inv_freq / factor, inv_freq)
        is_mid = (wl >= high_wl) & (wl <= low_wl)
        inv_freq = torch.where(is_mid, (1 - smooth) * inv_freq / factor + smooth * inv_freq, scaled)
    t = torch.arange(max_pos, dtype=torch.float64)
    freqs = torch.outer(t, inv_freq)
    return torch.cat([freqs.cos(), freqs.sin()], dim=-1).float().to(device)


def apply_rope(x: torch.Tensor, positions: torch.Tensor, cos_sin: torch.Tensor) -> torch.Tensor:
    """x [T, H, D] -> rotated (rotate-half convention), computed in fp32."""
    d2 = x.shape[-1] // 2
    cs = cos_sin[positions.long()]  # [T, D]
    cos, sin = cs[:, None, :d2], cs[:, None, d2:]
    xf = x.float()
    x1, x2 = xf[..., :d2], xf[..., d2:]
    return torch.cat([x1 * cos - x2 * sin, x2 * cos + x1 * sin], dim=-1).to(x.dtype)


FP8_KV = (torch.float8_e4m3fn, torch.uint8)
FP8_MAX = 448.0


def is_fp8_kv(kv: torch.Tensor) -> bool:
    return kv.dtype in FP8_KV


def write_kv(kv_layer: torch.Tensor, k: torch.Tensor, v: torch.Tensor, slot_mapping: torch.Tensor,
             k_scale: float = 1.0, v_scale: float = 1.0):
    """kv_layer [NB, 2, Hkv, BS, D]; k, v [T, Hkv, D].  An fp8 (e4m3fn) cache stores x / scale,
    saturated to +-448."""
    if is_fp8_kv(kv_layer):
        k = (k.float() / k_scale).clamp(-FP8_MAX, FP8_MAX).to(torch.float8_e4m3fn)
        v = (v.float() / v_scale).clamp(-FP8_MAX, FP8_MAX).to(torch.float8_e4m3fn)
        if kv_layer.dtype == torch.uint8:
            k, v = k.view(torch.uint8), v.view(torch.uint8)
    bs = kv_layer.shape[3]
    d = kv_layer.shape[4]
    valid = slot_mapping >= 0
    slots = slot_mapping[valid].long()
    if slots.numel() == 0:
        return
    blk, off = slots // bs, slots % bs
    kk, vv = k[valid], v[valid]
    for i in range(slots.numel()):
        b, o = int(blk[i]), int(off[i])
        kv_layer[b, 0, :, o, :] = kk[i]
        # V dim-major: view the [BS, D] region as [D, BS]
        kv_layer[b, 1].view(kv_layer.shape[2], d, bs)[:, :, o] = vv[i]


def rope_and_cache(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, positions: torch.Tensor,
                   cos_sin: torch.Tensor, kv_layer: torch.Tensor, slot_mapping: torch.Tensor,
                   q_norm_w: Optional[torch.Tensor] = None, k_norm_w: Optional[torch.Tensor] = None,
                   eps: float = 1e-6, k_scale: float = 1.0, v_scale: float = 1.0):
    """Optional per-head RMSNorm (Qwen3), RoPE on q/k, write k/v into the paged cache.
    q [T, Hq, D], k/v [T, Hkv, D].  Returns rotated q (new tensor)."""
    if q_norm_w is not None:
        q = rms_norm(q, q_norm_w, eps)
        k = rms_norm(k, k_norm_w, eps)
    q = apply_rope(q, positions, cos_sin)
    k = apply_rope(k, positions, cos_sin)
    write_kv(kv_layer, k, v, slot_mapping, k_scale, v_scale)
    return q


def gather_kv(kv_layer: torch.Tensor, block_table: torch.Tensor, n: int, k_scale: float = 1.0,
              v_scale: float = 1.0):
    """Return K, V [n, Hkv, D] for the first n tokens of a sequence (fp32, dequantised, for an fp8
    cache)."""
    if is_fp8_kv(kv_layer):
        K, V = _gather_raw(kv_layer.view(torch.uint8), block_table, n)
        f8 = torch.float8_e4m3fn
        return K.view(f8).float() * k_scale, V.view(f8).float() * v_scale
    return _gather_raw(kv_layer, block_table, n)


def _gather_raw(kv_layer: torch.Tensor, block_table: torch.Tensor, n: int):
    bs, d, hkv = kv_layer.shape[3], kv_layer.shape[4], kv_layer.shape[2]
    nb = (n + bs - 1) // bs
    blocks = block_table[:nb].long()
    kb = kv_layer[blocks, 0]  # [nb, Hkv, BS, D]
    vb = kv_layer[blocks, 1].reshape(nb, hkv, d, bs)  # dim-major
    K = kb.permute(0, 2, 1, 3).reshape(nb * bs, hkv, d)[:n]
    V = vb.permute(0, 3, 1, 2).reshape(nb * bs, hkv, d)[:n]
    return K, V


def _attend(q: torch.Tensor, K: torch.Tensor, V: torch.Tensor, q_pos0: int, scale: float):
    """q [m, Hq, D] (query positions q_pos0..q_pos0+m-1), K/V [n, Hkv, D]; causal."""
    m, hq, d = q.shape
    n, hkv = K.shape[0], K.shape[1]
    g = hq // hkv
    Kf = K.float().repeat_interleave(g, dim=1)  # [n, Hq, D]
    Vf = V.float().repeat_interleave(g, dim=1)
    s = torch.einsum("mhd,nhd->hmn", q.float(), Kf) * scale
    qpos = torch.arange(m, device=q.device).unsqueeze(1) + q_pos0
    kpos = torch.arange(n, device=q.device).unsqueeze(0)
    s = s.masked_fill((kpos > qpos).unsqueeze(0), float("-inf"))
    p = torch.softmax(s, dim=-1)
    return torch.einsum("hmn,nhd->mhd", p, Vf)


def paged_attention(q: torch.Tensor, kv_layer: torch.Tensor, block_tables: torch.Tensor,
                    query_start_loc: torch.Tensor, seq_lens: torch.Tensor, scale: float, k_scale: float = 1.0,
                    v_scale: float = 1.0) -> torch.Tensor:
    """Varlen causal attention over the paged cache (prefill chunks and decode alike).
    q [T, Hq, D]; sequence i owns q rows query_start_loc[i]:query_start_loc[i+1], whose positions
    are the LAST q_len positions of its seq_lens[i] tokens (cache already holds them)."""
    out = torch.empty(q.shape, dtype=torch.float32, device=q.device)
    qsl = query_start_loc.tolist()
    sl = seq_lens.tolist()
    for i in range(len(sl)):
        a, b = qsl[i], qsl[i + 1]
        if b <= a:
            continue
        K, V = gather_kv(kv_layer, block_tables[i], sl[i], k_scale, v_scale)
        out[a:b] = _attend(q[a:b], K, V, sl[i] - (b - a), scale)
    return out.to(q.dtype)


def paged_attention_decode(q, kv_layer, block_tables, seq_lens, scale, k_scale: float = 1.0, v_scale: float = 1.0):
    qsl = torch.arange(q.shape[0] + 1, dtype=torch.int32)
    return paged_attention(q, kv_layer, block_tables, qsl, seq_lens, scale, k_scale, v_scale)


# ----------------------------------------------------------------------------- sampling
def _hash_u32(x: torch.Tensor) -> torch.Tensor:
    """Counter-based integer hash (same mixing as csrc/kernels/sampling.hip: splitmix-style)."""
    x = x.to(torch.int64) & 0xFFFFFFFF
    x = ((x ^ (x >> 16)) * 0x7FEB352D) & 0xFFFFFFFF
    x = ((x ^ (x >> 15)) * 0x846CA68B) & 0xFFFFFFFF
    x = x ^ (x >> 16)
    return x


def uniform_noise(seeds: torch.Tensor, steps: torch.Tensor, vocab: int) -> torch.Tensor:
    """u[b, v] in (0,1) from (seed, step, v): deterministic per request (reproducible sampling)."""
    b = seeds.shape[0]
    idx = torch.arange(vocab, dtype=torch.int64).unsqueeze(0).expand(b, vocab)
    key = _hash_u32(seeds.to(torch.int64).unsqueeze(1) * 0x9E3779B1 + steps.to(torch.int64).unsqueeze(1))
    h = _hash_u32(key ^ _hash_u32(idx + 0x632BE5AB))
    return ((h >> 8).double() + 0.5) / float(1 << 24)


def sample(logits: torch.Tensor, temperature: torch.Tensor, top_p: torch.Tensor, top_k: torch.Tensor,
           seeds: torch.Tensor, steps: torch.Tensor) -> torch.Tensor:
    """Per-row: temperature<=0 -> argmax.  Else Gumbel-max over the top-k / top-p nucleus of
    softmax(logits / T).  Returns int64 token ids [B]."""
    lf = logits.float()
    B, V = lf.shape
    out = torch.empty(B, dtype=torch.int64)
    u = uniform_noise(seeds.cpu(), steps.cpu(), V).to(lf.device)
    for i in range(B):
        t = float(temperature[i])
        row = lf[i]
        if t <= 0.0:
            out[i] = int(torch.argmax(row))
            continue
        z = row / t
        keep = torch.ones(V, dtype=torch.bool, device=lf.device)
        k = int(top_k[i])
        if 0 < k < V:
            kth = torch.topk(z, k).values[-1]
            keep &= z >= kth
        p = float(top_p[i])
        if p < 1.0:
            probs = torch.softmax(z, -1)
            sp, si = torch.sort(probs, descending=True)
            csum = torch.cumsum(sp, 0)
            # smallest prefix with mass >= p ; threshold = prob of the last kept element
            n_keep = int((csum < p).sum()) + 1
            thr = sp[min(n_keep, V) - 1]
            keep &= probs >= thr
        g = -torch.log(-torch.log(u[i].float()))
        score = torch.where(keep, z + g, torch.full_like(z, float("-inf")))
        out[i] = int(torch.argmax(score))
    return out.to(logits.device)


def apply_penalties(logits, hist, srows, hlen, plen, rep, freq, pres) -> torch.Tensor:
    """In place: repetition penalty over prompt + generated tokens, frequency / presence penalties
    over generated tokens (history hist[row, :hlen], the first plen entries being the prompt)."""
    for b in range(logits.shape[0]):
        rp, fp, pp = float(rep[b]), float(freq[b]), float(pres[b])
        if rp == 1.0 and fp == 0.0 and pp == 0.0:
            continue
        V = logits.shape[1]
        h = hist[int(srows[b]), :int(hlen[b])].long().cpu()
        np_ = min(int(plen[b]), len(h))
        counts = torch.bincount(h[np_:].clamp(0, V - 1), minlength=V).to(logits.device)
        seen = counts > 0
        if np_:
            seen[h[:np_].clamp(0, V - 1).to(logits.device)] = True
        z = logits[b].float()
        if rp != 1.0:
            z = torch.where(seen, torch.where(z > 0, z / rp, z * rp), z)
        z = z - counts.float() * fp - (counts > 0).float() * pp
        logits[b] = z.to(logits.dtype)
    return logits


def logprobs(logits: torch.Tensor, rows: torch.Tensor, tokens: torch.Tensor, k: int):
    """Raw-distribution log-probs: the sampled token's, and the k best (value desc, index asc)."""
    lp = torch.log_softmax(logits.index_select(0, rows.long()).float(), dim=-1)
    tok_lp = lp.gather(1, tokens.long().view(-1, 1)).squeeze(1)
    if k == 0:
        return tok_lp, torch.zeros(len(rows), 0, dtype=torch.int64), torch.zeros(len(rows), 0)
    # stable order on ties: sort by index first, then a stable sort by value
    order = torch.sort(lp, dim=-1, descending=True, stable=True)
    return tok_lp, order.indices[:, :k].contiguous(), order.values[:, :k].contiguous()


# ----------------------------------------------------------------------------- MoE
def moe_topk_softmax(router_logits: torch.Tensor, k: int, renormalize: bool = True):
    probs = torch.softmax(router_logits.float(), dim=-1)
    w, ids = torch.topk(probs, k, dim=-1)
    if renormalize:
        w = w / w.sum(-1, keepdim=True)
    return w, ids.to(torch.int32)


def moe_experts(x: torch.Tensor, w13: torch.Tensor, w2: torch.Tensor, topk_w: torch.Tensor,
                topk_ids: torch.Tensor, expert_offset: int = 0) -> torch.Tensor:
    """x [T, H]; w13 [E_local, 2I, H]; w2 [E_local, H, I]; returns sum_k w_k * expert_k(x) for
    experts owned locally (global id - expert_offset in [0, E_local))."""
    T, H = x.shape
    out = torch.zeros(T, H, dtype=torch.float32, device=x.device)
    e_local = w13.shape[0]
    for e in range(e_local):
        mask = topk_ids == (e + expert_offset)
        tok, slot = mask.nonzero(as_tuple=True)
        if tok.numel() == 0:
            continue
        h = x[tok].float() @ w13[e].float().t()
        a = silu_mul(h)
        y = a @ w2[e].float().t()
        out.index_add_(0, tok, y * topk_w[tok, slot].unsqueeze(1).float())
    return out.to(x.dtype)
