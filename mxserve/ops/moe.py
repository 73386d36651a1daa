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

import bisect
import logging
import os
import time

import torch
import torch.nn.functional as F

log = logging.getLogger(__name__)

DENSE_MAX_TOKENS = 256
# decode batches (T tokens <= this, graph-captured): both expert GEMMs on the grouped form of the
# decode GEMM kernel (gemm_decode.hip: weights streamed through registers, wave tile sized to the
# few rows each expert gets) instead of the 128-row LDS tiles of moe_gemm.hip
DECODE = os.environ.get("MXS_MOE_DECODE_GEMM", "1") != "0"
DECODE_MAX_TOKENS = 256
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
    inv = torch.empty(T * K, dtype=torch.int32, device=x.device)
    ext().moe_align(offs, perm, ids, expert_offset, e_local, inv)
    o = offs.tolist()  # prefill runs eagerly: one host sync for the per-expert slices
    x = x.contiguous()
    xs = torch.empty(max(o[-1], 1), H, dtype=x.dtype, device=x.device)
    ext().ep_gather_rows(xs, x, inv, K)  # xs[inv[p]] = x[p // K]
    ys = torch.empty(max(o[-1], 1), H, dtype=x.dtype, device=x.device)
    for e in range(e_local):
        a, b = o[e], o[e + 1]
        if b > a:
            ys[a:b] = F.linear(_silu_mul(F.linear(xs[a:b], w13[e])), w2[e])
    out = torch.empty(T, H, dtype=x.dtype, device=x.device)
    ext().moe_combine(out, ys, topk_w.float().contiguous(), inv)  # K17: weighted sum, fp32, one write
    return out


# measured at graph capture (tune()): (H, I, E_local, top_k) -> sorted [(T bucket, cfg13, cfg2)];
# cfg13 None = the LDS-tiled grouped GEMM measured faster for that bucket
TABLE: dict = {}


def _table_cfg(T: int, H: int, I: int, e_local: int, top_k: int):
    ent = TABLE.get((H, I, e_local, top_k))
    if not ent:
        return False
    i = bisect.bisect_left(ent, (T,))
    if i == len(ent):
        return None
    return ent[i][1], ent[i][2]


def decode_cfg(T: int, N: int, K: int, epi: int, e_local: int, top_k: int = 2) -> tuple | None:
    """Untuned default (mf, nf, wm, splitk) of the grouped decode kernel for T tokens: the wave's row
    tile covers the average rows per expert (T * top_k / experts), enough split-K to put ~1024
    workgroups on the chip.  tune() replaces it per bucket with measured choices
    (scripts/moe_decode_probe.py prints every configuration)."""
    from .decode_gemm import unroll
    avg = -(-T * top_k // max(1, e_local))
    mf = 1 if avg <= 16 else (2 if avg <= 32 else 4)
    nf = 2 if epi else 4
    nh = nf // 2 if epi else nf
    out_n = N // 2 if epi else N
    bn = 4 * nh * 16
    if out_n % bn:
        return None
    tiles = (out_n // bn) * min(e_local, T * top_k)
    best = None
    for sk in (1, 2, 4, 8):
        if K % (32 * unroll(mf, nf) * sk) == 0:
            best = (mf, nf, 1, sk, 0)
            if tiles * sk >= 1024:
                break
    return best


# split-K slices the fused epilogues (silu_mul_partials, moe_combine_partials) sum at most
MAX_SLABS = 8


def _mdg(out, x, w, offs, part, rows_max: int, cfg: tuple, epi: int) -> bool:
    from . import ext
    mf, nf, wm, sk = cfg[:4]
    return bool(ext().moe_decode_gemm(out, x, w, offs, part, rows_max, mf, nf, wm, sk, epi,
                                      cfg[4] if len(cfg) > 4 else 0))


def _fused_experts_decode(x, w13, w2, topk_w, offs, inv, xs, expert_offset) -> torch.Tensor | None:
    from . import ext
    T, H = x.shape
    K = topk_w.shape[1]
    e_local, two_i, _ = w13.shape
    R = T * K
    tuned = _table_cfg(T, H, two_i // 2, e_local, K)
    if tuned is False:  # not tuned for this shape: defaults
        c13 = decode_cfg(T, two_i, H, 1, e_local, K)
        c2 = decode_cfg(T, H, two_i // 2, 0, e_local, K)
    elif tuned is None:
        return None
    else:
        c13, c2 = tuned
    if c13 is None or c2 is None or c13[3] > MAX_SLABS or c2[3] > MAX_SLABS:
        return None
    dev = x.device
    h = torch.empty(R, two_i // 2, dtype=x.dtype, device=dev)
    if c13[3] > 1:
        p13 = torch.empty(c13[3], R, two_i, dtype=torch.float32, device=dev)
        if not _mdg(h, xs, w13, offs, p13, T, c13, 1):
            return None
        ext().silu_mul_partials(h, p13)
    elif not _mdg(h, xs, w13, offs, None, T, c13, 1):
        return None
    out = torch.empty(T, H, dtype=x.dtype, device=dev)
    tw = topk_w.float().contiguous()
    if c2[3] > 1:
        p2 = torch.empty(c2[3], R, H, dtype=torch.float32, device=dev)
        if not _mdg(h, h, w2, offs, p2, T, c2, 0):
            return None
        ext().moe_combine_partials(out, p2, tw, inv)
    else:
        ys = torch.empty(R, H, dtype=x.dtype, device=dev)
        if not _mdg(ys, h, w2, offs, None, T, c2, 0):
            return None
        ext().moe_combine(out, ys, tw, inv)
    return out


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
    perm = torch.empty(T * K, dtype=torch.int32, device=dev)
    inv = torch.empty(T * K, dtype=torch.int32, device=dev)
    ext().moe_align(offs, perm, ids, expert_offset, e_local, inv)
    # xs[inv[p]] = x[p // K] in one kernel; rows past the routed count stay unset (never read as data)
    x = x.contiguous()
    xs = torch.empty(T * K, H, dtype=x.dtype, device=dev)
    ext().ep_gather_rows(xs, x, inv, K)
    if DECODE and T <= DECODE_MAX_TOKENS and w13.is_contiguous() and w2.is_contiguous():
        out = _fused_experts_decode(x, w13, w2, topk_w, offs, inv, xs, expert_offset)
        if out is not None:
            return out
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


def tune(w13: torch.Tensor, w2: torch.Tensor, buckets: list, top_k: int, n_experts: int, expert_offset: int = 0,
         device=None) -> list:
    """Per decode bucket T: time every configuration of the grouped decode kernel for both expert
    GEMMs (hipGraph-replayed, synthetic uniform routing over all n_experts), then the whole layer
    on the tuned kernel vs the LDS-tiled grouped GEMM, and keep the faster (TABLE).  Returns the
    report rows."""
    global DECODE
    from . import ext
    from .decode_gemm import _graph_time, candidates
    if not DECODE:
        return []
    e_local, two_i, H = w13.shape
    I = two_i // 2
    dev = device or w13.device
    g = torch.Generator(device=dev).manual_seed(0)
    bks = sorted(b for b in buckets if b <= DECODE_MAX_TOKENS)
    t0 = time.time()
    rows, ent = [], []
    key = (H, I, e_local, top_k)
    TABLE.pop(key, None)
    from .tuned import TunedStore, device_tag
    store = TunedStore("moe_decode", device_tag(dev))
    for T in bks:
        R = T * top_k
        x = torch.randn(T, H, device=dev, generator=g).to(w13.dtype)
        logits = torch.randn(T, n_experts, device=dev, generator=g)
        tw, ids = torch.topk(torch.softmax(logits, -1), top_k, dim=-1)
        tw, ids = (tw / tw.sum(-1, keepdim=True)).float().contiguous(), ids.to(torch.int32).contiguous()
        offs = torch.empty(e_local + 1, dtype=torch.int32, device=dev)
        perm = torch.full((R,), -1, dtype=torch.int32, device=dev)
        inv = torch.empty(R, dtype=torch.int32, device=dev)
        ext().moe_align(offs, perm, ids, expert_offset, e_local, inv)
        xs = x.index_select(0, perm.clamp(min=0).long() // top_k)
        h = torch.empty(R, I, dtype=w13.dtype, device=dev)
        ys = torch.empty(R, H, dtype=w13.dtype, device=dev)
        part = torch.empty(8 * R * max(two_i, H), dtype=torch.float32, device=dev)
        skey = f"{H}x{I}x{e_local}x{top_k}x{n_experts}@{T}"
        st = store.get(skey)
        if st is not None:  # persisted choice: only the correctness check below runs
            cfg = st.get("cfg") or (None, None)
            if not st.get("use") or cfg[0] is None or cfg[1] is None:
                ent.append((T, None, None))
                rows.append({"T": T, "chosen": "grouped_lds", "source": "table"})
                continue
            DECODE = False
            ref = fused_experts(x, w13, w2, tw, ids, expert_offset)
            DECODE = True
            TABLE[key] = ent + [(T, cfg[0], cfg[1])]
            out = fused_experts(x, w13, w2, tw, ids, expert_offset)
            err = (out.float() - ref.float()).abs().max().item()
            ok = err <= 0.03 * max(1.0, ref.float().abs().max().item())
            ent.append((T, cfg[0], cfg[1]) if ok else (T, None, None))
            rows.append({"T": T, "cfg_w13": cfg[0], "cfg_w2": cfg[1], "chosen": "decode" if ok else "grouped_lds",
                         "max_abs_err": err, "source": "table"})
            continue
        best = {}
        for name, w, epi, N, K, o, xin in (("w13", w13, 1, two_i, H, h, xs), ("w2", w2, 0, H, I, ys, h)):
            bt, bc = None, None
            for cfg in candidates(T, N, K, epi, all_mf=True, mt=False):
                sk = cfg[3]
                if cfg[2] > 2 or sk > MAX_SLABS:  # the slab-summing epilogues take at most 8 slices
                    continue
                pp = part[: sk * R * N].view(sk, R, N) if sk > 1 else None
                if not _mdg(o, xin, w, offs, pp, T, cfg, epi):
                    continue
                t = _graph_time(lambda: _mdg(o, xin, w, offs, pp, T, cfg, epi))
                if bt is None or t < bt:
                    bt, bc = t, cfg
            best[name] = bc
        if best["w13"] is None or best["w2"] is None:
            ent.append((T, None, None))
            continue
        DECODE = False
        t_lds = _graph_time(lambda: fused_experts(x, w13, w2, tw, ids, expert_offset))
        ref = fused_experts(x, w13, w2, tw, ids, expert_offset)
        DECODE = True
        TABLE[key] = ent + [(T, best["w13"], best["w2"])]
        t_dec = _graph_time(lambda: fused_experts(x, w13, w2, tw, ids, expert_offset))
        out = fused_experts(x, w13, w2, tw, ids, expert_offset)
        err = (out.float() - ref.float()).abs().max().item()
        ok = err <= 0.03 * max(1.0, ref.float().abs().max().item())
        use = ok and t_dec < t_lds * 0.98
        store.put(skey, {"cfg": (best["w13"], best["w2"]), "use": bool(use), "layer_decode_us": round(t_dec, 1),
                         "layer_grouped_lds_us": round(t_lds, 1)})
        ent.append((T, best["w13"], best["w2"]) if use else (T, None, None))
        rows.append({"T": T, "cfg_w13": best["w13"], "cfg_w2": best["w2"], "layer_decode_us": round(t_dec, 1),
                     "layer_grouped_lds_us": round(t_lds, 1), "chosen": "decode" if use else "grouped_lds",
                     "max_abs_err": err})
    TABLE[key] = ent
    store.save()
    path = os.environ.get("MXS_MOE_GEMM_REPORT")
    if path:
        import json
        with open(path, "w") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")
    log.info("MoE decode GEMM tuning: decode kernel chosen for %d of %d buckets in %.1fs",
             sum(r["chosen"] == "decode" for r in rows), len(bks), time.time() - t0)
    return rows
