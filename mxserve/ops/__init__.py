"""Op registry: one entry point per engine op.

GPU tensors go to the hand-written gfx950 HIP kernels in the in-tree extension `mxserve/_C*.so`
(built by `python setup_ext.py` / `__graft_entry__.build()`); CPU tensors go to the PyTorch
reference in `reference.py`.  A GPU tensor with no extension loaded is an error, never a silent
fallback (the driver checks which `.so` files the GPU tests load).
"""
from __future__ import annotations

import importlib
import os
from typing import Optional

import torch

from . import reference as ref

_EXT = None
_EXT_ERR: Optional[BaseException] = None


def ext():
    """Load (once) and return the native HIP extension module."""
    global _EXT, _EXT_ERR
    if _EXT is None and _EXT_ERR is None:
        try:
            _EXT = importlib.import_module("mxserve._C")
        except BaseException as e:  # noqa: BLE001 - re-raised on first GPU use
            _EXT_ERR = e
    if _EXT is None:
        raise RuntimeError(
            "mxserve HIP extension (mxserve/_C*.so) is not built or failed to load: "
            f"{_EXT_ERR!r}. Run `python setup_ext.py` (hipcc --offload-arch=gfx950).")
    return _EXT


def has_ext() -> bool:
    try:
        ext()
        return True
    except RuntimeError:
        return False


# ----------------------------------------------------------------------------- IPC
# hipIpcOpenMemHandle of a peer GPU's allocation can hang for some sizes (measured r1:
# profiles/r1_ipc_open_probe.txt; disagg/kv_transfer.py module docstring).  Every open goes through
# ipc_open(): a deadline, after which IPC is marked broken for this process (the stuck call still
# holds the native table's lock) and callers fall back -- the KV transfer to the /dev/shm arena or
# HTTP, the TP all-reduce to RCCL.
IPC_STATE: dict = {"broken": None}


def ipc_open(handle: bytes, offset: int = 0, timeout_s: Optional[float] = None) -> int:
    """Map a peer's exported allocation (comm.cpp open_pool) within timeout_s seconds (default
    MXS_IPC_OPEN_TIMEOUT_S, 30); raises TimeoutError (an OSError) past it and on every later call."""
    import threading
    if IPC_STATE["broken"]:
        raise TimeoutError(f"IPC disabled in this process: {IPC_STATE['broken']}")
    timeout_s = float(os.environ.get("MXS_IPC_OPEN_TIMEOUT_S", "30")) if timeout_s is None else timeout_s
    box: dict = {}
    done = threading.Event()
    fn = ext().ipc_open_pool

    def run():
        try:
            box["ptr"] = int(fn(handle, int(offset)))
        except BaseException as e:  # noqa: BLE001 - re-raised in the caller
            box["err"] = e
        finally:
            done.set()
    threading.Thread(target=run, name="mxs-ipc-open", daemon=True).start()  # daemon: a hung open never blocks exit
    if not done.wait(timeout_s):
        IPC_STATE["broken"] = f"hipIpcOpenMemHandle did not return within {timeout_s:.0f}s"
        raise TimeoutError(IPC_STATE["broken"])
    if "err" in box:
        raise box["err"]
    return box["ptr"]


_PREFILL_VERSION = int(os.environ.get("MXS_PREFILL_KERNEL", "3"))


_DECODE_IMPL = int(os.environ.get("MXS_DECODE_ATTN", "0"))


def _gpu(t: torch.Tensor) -> bool:
    return t.is_cuda and os.environ.get("MXS_FORCE_REFERENCE_OPS", "0") != "1"


# ----------------------------------------------------------------------------- GEMM
def linear(x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """y = x @ w.T.  Decode-sized GEMMs (M <= decode_gemm.MAX_M) run the hand-written MFMA kernel where the
    tuning pass at graph capture measured it faster than hipBLASLt for that batch bucket and
    projection (mxserve/ops/decode_gemm.py); everything else is hipBLASLt."""
    if _gpu(x) and x.dim() == 2:
        M = x.shape[0]
        from . import decode_gemm
        if M <= decode_gemm.MAX_M:
            cfg = decode_gemm.TABLE.lookup(M, w.shape[0], w.shape[1], 0)
            if cfg is not None:
                out = torch.empty(M, w.shape[0], dtype=x.dtype, device=x.device)
                if decode_gemm.TABLE.run(out, x, w, cfg, 0):
                    return out
        if M > 256:
            # prefill chunks: the persistent stream-K MFMA kernel where the start-up tuner measured it
            # faster (ops/prefill_pf.py)
            from .prefill_pf import TABLE as PF_TABLE, pf_cfg
            mi = PF_TABLE.lookup(M, w.shape[0], w.shape[1], 0)
            if mi is not None:
                it, tr = pf_cfg(mi)
                out = gemm_pf(x, w, 0, None, it, trows=tr)
                if out is not None:
                    return out
            # small prefill chunks: the 64/128-row tile kernel where it was measured faster
            from .decode_gemm import PREFILL_TABLE
            cfg = PREFILL_TABLE.lookup(M, w.shape[0], w.shape[1])
            if cfg is not None:
                out = torch.empty(M, w.shape[0], dtype=x.dtype, device=x.device)
                if prefill_gemm(out, x, w, cfg):
                    return out
            # hipBLASLt with the solution measured fastest for this bucket (ops/prefill_hblt.py)
            from . import prefill_hblt
            out = prefill_hblt.linear(x, w)
            if out is not None:
                return out
            plan = _mplan(M, w.shape[0], w.shape[1], x.device)
            if plan is not None:
                return _run_mplan(x, w, plan)
    return torch.nn.functional.linear(x, w)


# ----------------------------------------------------------------------------- prefill M plans
# hipBLASLt's kernel choice is not monotone in the row count: Llama-3.2-1B gate_up takes 189 us at
# 4096 rows and 247 us at 4224-4352 (a mixed step with one 4000-token prompt and ~270 decode rows),
# down 171 us at 8192 and 396 us at 8320; F.linear and mm(out=) sometimes pick different kernels too
# (profiles/r3/s3/hipblaslt_m_sweep.jsonl, 128-row grid).  A persisted per-device plan
# (ops/tuned/prefill_mplan_<arch>_<cus>cu.json, built from that sweep) splits such a GEMM into a
# sweet-spot block plus the remainder, or takes the faster call form, wherever that measured >= 4 %
# faster than one F.linear.  MXS_MPLAN=0 disables.
_MPLAN: dict = {}


def _mplan(M: int, N: int, K: int, device) -> Optional[list]:
    if os.environ.get("MXS_MPLAN", "1") != "1":
        return None
    tab = _MPLAN.get(device)
    if tab is None:
        tab = _MPLAN[device] = _load_mplan(device)
    ent = tab.get(f"{N}x{K}")
    if not ent:
        return None
    # each shape's entry lives on the row grid it was swept on (the packaged table: 128 rows; start-up
    # tuning: 256): the grid is its smallest bucket.  Only that grid's bucket is looked up -- a plan
    # measured for the next coarser bucket must not be stretched over up to 255 shaved rows
    g = ent.get("_grid")
    if g is None:
        g = ent["_grid"] = min(int(k) for k in ent if k.isdigit())
    bucket = -(-M // g) * g
    e = ent.get(str(bucket))
    if e is None:
        return None
    plan = [list(seg) for seg in e["plan"]]
    short = bucket - M
    if short:  # the actual rows are up to 127 fewer than the bucket: take them off the smaller segment
        i = min(range(len(plan)), key=lambda j: plan[j][0])
        if plan[i][0] <= short:
            return None
        plan[i][0] -= short
    return plan


def _load_mplan(device) -> dict:
    from .mplan import load
    return load(device)


def _run_mplan(x: torch.Tensor, w: torch.Tensor, plan: list) -> torch.Tensor:
    M = x.shape[0]
    if len(plan) == 1 and plan[0][1] == "lin":
        return torch.nn.functional.linear(x, w)
    y = torch.empty(M, w.shape[0], dtype=x.dtype, device=x.device)
    r = 0
    for rows, form in plan:
        xs, ys = x[r:r + rows], y[r:r + rows]
        if form == "mm":
            torch.mm(xs, w.t(), out=ys)
        else:
            ys.copy_(torch.nn.functional.linear(xs, w))
        r += rows
    assert r == M, (r, M, plan)
    return y


_PG_PART: dict = {}


def _decode_max_m() -> int:
    from .decode_gemm import MAX_M
    return MAX_M


def prefill_gemm_configs(M: int, N: int, K: int) -> list:
    """(bm, splitk) configurations of the prefill GEMM kernel (csrc/kernels/gemm_prefill.hip)."""
    if N % 128:
        return []
    return [(bm, sk) for bm in (64, 128) for sk in (1, 2, 4) if K % (64 * sk) == 0]


def prefill_gemm(out: torch.Tensor, x: torch.Tensor, w: torch.Tensor, cfg: tuple) -> bool:
    bm, sk = cfg
    part = None
    if sk > 1:
        need = sk * x.shape[0] * w.shape[0]
        part = _PG_PART.get(x.device)
        if part is None or part.numel() < need:
            part = _PG_PART[x.device] = torch.empty(need, dtype=torch.float32, device=x.device)
    return bool(ext().prefill_gemm(out, x, w, part, bm, sk))


# ----------------------------------------------------------------------------- prefill GEMM (gemm_pf.hip)
_PF_WS: dict = {}


def _pf_workspace(device) -> tuple:
    """(fp32 stream-K slabs, int32 tile counters, CU count) of a device; the counters start zero and
    every launch leaves them zero."""
    ws = _PF_WS.get(device)
    if ws is None:
        ncu = torch.cuda.get_device_properties(device).multi_processor_count
        slab = torch.empty(2 * ncu * 34 * 512 * 4, dtype=torch.float32, device=device)  # PF_SLAB_FRAGS = 34
        cnt = torch.zeros(1 << 16, dtype=torch.int32, device=device)
        ws = _PF_WS[device] = (slab, cnt, ncu)
    return ws


def gemm_pf_faults(device=None) -> int:
    """Stream-K tile heads of gemm_pf whose wait for the tile's other segments timed out since the
    workspace was made (csrc/kernels/gemm_pf.hip: the counters' last word).  Non-zero means a launch
    ran while its grid was not fully resident (another process holding CUs) and produced wrong sums
    for those tiles; the engine reports it in stats() and the GPU tests require zero."""
    dev = torch.device(device) if device is not None else torch.device("cuda")
    if dev.index is None:
        dev = torch.device(dev.type, torch.cuda.current_device())
    ws = _PF_WS.get(dev)
    return 0 if ws is None else int(ws[1][-1].item())


_HBLT_WS: dict = {}
HBLT_WS_BYTES = 64 << 20  # hipBLASLt stream-K solutions' workspace


def _hblt_ws(device) -> torch.Tensor:
    ws = _HBLT_WS.get(device)
    if ws is None:
        ws = _HBLT_WS[device] = torch.empty(HBLT_WS_BYTES, dtype=torch.uint8, device=device)
    return ws


def hblt_candidates(M: int, N: int, K: int, resid: bool = False, heuristic: int = 8) -> list:
    """hipBLASLt solution indices that support x [M, K] @ w [N, K].T (+ a residual, beta 1): the
    library heuristic's top `heuristic` first, then every other supporting gfx950 solution
    (csrc/kernels/hblt.cpp)."""
    return list(ext().hblt_candidates(M, N, K, resid, heuristic, HBLT_WS_BYTES))


def hblt_mm(x: torch.Tensor, w: torch.Tensor, index: int, out: Optional[torch.Tensor] = None,
            resid: Optional[torch.Tensor] = None) -> Optional[torch.Tensor]:
    """out = x @ w.T (+ resid; out may be resid: in place) with hipBLASLt solution `index`; None when
    that solution does not support the shape (the caller takes the default path)."""
    if out is None:
        out = torch.empty(x.shape[0], w.shape[0], dtype=x.dtype, device=x.device)
    if not ext().hblt_mm(out, x, w, resid, int(index), _hblt_ws(x.device)):
        return None
    return out


_PF_FAULT_HOST: dict = {}


def gemm_pf_faults_async(device=None) -> int:
    """gemm_pf_faults() without a device sync, for callers on a serving loop (AsyncEngine reads the
    engine's stats every 20 ms; an .item() there drained the queue the host had run ahead with): the
    word is copied into pinned memory behind the work already queued, and each call returns the
    latest copy that has landed (0 before the first)."""
    dev = torch.device(device) if device is not None else torch.device("cuda")
    if dev.index is None:
        dev = torch.device(dev.type, torch.cuda.current_device())
    ws = _PF_WS.get(dev)
    if ws is None:
        return 0
    ent = _PF_FAULT_HOST.get(dev)
    if ent is None:
        ent = _PF_FAULT_HOST[dev] = [torch.zeros(1, dtype=torch.int32, pin_memory=True), None, 0]
    buf, ev, last = ent
    if ev is not None and not ev.query():
        return last  # the previous copy is still behind queued work
    if ev is not None:
        ent[2] = last = int(buf[0])
    buf.copy_(ws[1][-1:], non_blocking=True)
    ent[1] = ev = torch.cuda.Event()
    ev.record()
    return last


_PF_MAPS: dict = {}


def pf_tile_map(ntm: int, ntn: int, device, gm: int = 8) -> torch.Tensor:
    """Logical tile -> token tile | weight tile << 16 for gemm_pf: GM token tiles per weight-column
    sweep, so the 32 consecutive tiles an XCD runs together share W and X panels (cached)."""
    key = (ntm, ntn, gm, str(device))
    t = _PF_MAPS.get(key)
    if t is None:
        L = torch.arange(ntm * ntn, dtype=torch.int64)
        per = gm * ntn
        grp = L // per
        first = grp * gm
        gsz = torch.clamp(ntm - first, max=gm)
        ing = L - grp * per
        tm, tn = first + ing % gsz, ing // gsz
        t = _PF_MAPS[key] = (tm | (tn << 16)).to(torch.int32).to(device)
    return t


def gemm_w4(x: torch.Tensor, w: torch.Tensor, epi: int = 0, out: Optional[torch.Tensor] = None,
            resid: Optional[torch.Tensor] = None) -> Optional[torch.Tensor]:
    """Prefill GEMM, four-wave form (csrc/kernels/gemm_w4.hip: 128 x 128 per wave, data-parallel
    persistent): epi 0 x @ w.T, epi 1 SwiGLU over w = [gate; up], epi 2 resid + x @ w.T (out may be
    resid).  None when the shape is not supported (N % 256, K % 64)."""
    M, K = x.shape
    N = w.shape[0]
    if M == 0 or N % 256 or K % 64 or w.shape[1] != K:
        return None
    if out is None:
        out = torch.empty(M, N // 2 if epi == 1 else N, dtype=x.dtype, device=x.device)
    ncu = _pf_workspace(x.device)[2]
    if not ext().gemm_w4(out, x, w, epi, ncu, resid):
        return None
    return out


def gemm_pf(x: torch.Tensor, w: torch.Tensor, epi: int = 0, out: Optional[torch.Tensor] = None,
            min_iters: int = 16, resid: Optional[torch.Tensor] = None, row_scale: bool = False,
            eps: float = 1e-5, trows: int = 256) -> Optional[torch.Tensor]:
    """Prefill GEMM on the hand-written persistent stream-K kernel: epi 0 x @ w.T, epi 1 SiLU(x @
    gate.T) * (x @ up.T) with w = [gate; up], epi 2 resid + x @ w.T (out may be resid: in place).
    row_scale (epi 0 / 1): every row of the product is scaled by rsqrt(mean(x_row^2) + eps), i.e.
    RMSNorm(x) @ w'.T with the norm weight folded into w' (fold_norm_weight).  None when the shape is
    not supported.  trows: token-tile height (256, 224, 192, 160, 128): fewer rows per tile fill the CUs
    better when a 256-row tiling leaves a partial last round (e.g. 6,656 rows x 2,048 columns: 208
    tiles of 256 rows on 256 CUs, 240 of 224... 256 of 128 would be one full round at half the work
    per tile)."""
    M, N = x.shape[0], w.shape[0]
    if N % 256:
        return None
    if out is None:
        out = torch.empty(M, N // 2 if epi == 1 else N, dtype=x.dtype, device=x.device)
    slab, cnt, ncu = _pf_workspace(x.device)
    tmap = pf_tile_map(-(-M // trows), N // 256, x.device)
    if not ext().gemm_pf(out, x, w, epi, slab, cnt, tmap, ncu, min_iters, resid, row_scale, eps, trows):
        return None
    return out


def fold_norm_weight(w: torch.Tensor, norm_w: torch.Tensor) -> torch.Tensor:
    """w diag(norm_w): the weight a row-scaled GEMM (gemm_pf row_scale) multiplies by, so that
    rstd(x) * (x @ fold.T) == RMSNorm(x, norm_w) @ w.T."""
    return (w.float() * norm_w.float()[None, :]).to(w.dtype).contiguous()


def gate_up_silu(x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """silu(x @ gate.T) * (x @ up.T) with w = [gate; up] (K07 + K10).  Decode-sized: one MFMA kernel
    with SiLU*mul in its epilogue when tuned faster; prefill-sized: the stream-K kernel with the same
    epilogue (ops/prefill_pf.py); otherwise hipBLASLt + the SiLU*mul kernel."""
    if _gpu(x) and x.dim() == 2 and x.shape[0] > _decode_max_m():
        from .prefill_pf import TABLE as PF_TABLE, pf_cfg
        mi = PF_TABLE.lookup(x.shape[0], w.shape[0], w.shape[1], 1)
        if mi is not None:
            it, tr = pf_cfg(mi)
            out = gemm_pf(x, w, 1, None, it, trows=tr)
            if out is not None:
                return out
    if _gpu(x) and x.dim() == 2 and x.shape[0] <= _decode_max_m():
        from .decode_gemm import TABLE
        cfg = TABLE.lookup(x.shape[0], w.shape[0], w.shape[1], 1)
        if cfg is not None:
            out = torch.empty(x.shape[0], w.shape[0] // 2, dtype=x.dtype, device=x.device)
            if TABLE.run(out, x, w, cfg, 1):
                return out
    return silu_mul(linear(x, w))


# ----------------------------------------------------------------------------- norms / act
def rms_norm(x: torch.Tensor, w: torch.Tensor, eps: float) -> torch.Tensor:
    if _gpu(x):
        out = torch.empty_like(x)
        ext().rms_norm(out, x, w, eps)
        return out
    return ref.rms_norm(x, w, eps)


def fused_add_rms_norm(x: torch.Tensor, residual: torch.Tensor, w: torch.Tensor, eps: float):
    """Returns (normed, new_residual).  On GPU new_residual is `residual` updated in place."""
    if _gpu(x):
        out = torch.empty_like(x)
        ext().fused_add_rms_norm(out, x, residual, w, eps)
        return out, residual
    return ref.fused_add_rms_norm(x, residual, w, eps)


def linear_add_rms_norm(x: torch.Tensor, w: torch.Tensor, residual: torch.Tensor, norm_w: torch.Tensor,
                        eps: float):
    """(RMSNorm(residual + x @ w.T) * norm_w, residual updated in place) for a projection that feeds
    the residual stream (o_proj, down_proj; TP = 1).  When the decode table runs this projection
    split-K, the fp32 slabs go straight into one epilogue kernel (sum + add + norm) instead of the
    split-K reduce kernel, a bf16 output and the fused add + RMSNorm kernel."""
    if _gpu(x) and x.dim() == 2 and 0 < x.shape[0] <= _decode_max_m():
        from .decode_gemm import TABLE
        M, N = x.shape[0], w.shape[0]
        cfg = TABLE.lookup(M, N, w.shape[1], 0)
        if cfg is not None and TABLE.splitk(cfg) > 1:
            dummy = residual  # [M, N] bf16: the kernel writes no output when the reduce is skipped
            if TABLE.run(dummy, x, w, cfg, 0, reduce=False):
                out = torch.empty_like(residual)
                ext().splitk_add_rms_norm(out, residual, TABLE.part, TABLE.splitk(cfg), norm_w, eps)
                return out, residual
    return fused_add_rms_norm(linear(x, w), residual, norm_w, eps)


def embed_rms_norm(ids: torch.Tensor, table: torch.Tensor, w: torch.Tensor, eps: float):
    """Embedding gather fused with the first layer's input RMSNorm: returns (normed, residual)
    where residual = table[ids]."""
    if _gpu(table):
        T, H = ids.shape[0], table.shape[1]
        out = torch.empty(T, H, dtype=table.dtype, device=table.device)
        res = torch.empty(T, H, dtype=table.dtype, device=table.device)
        ext().embed_rms_norm(out, res, ids, table, w, eps)
        return out, res
    x = torch.nn.functional.embedding(ids, table)
    return ref.rms_norm(x, w, eps), x


def silu_mul(gu: torch.Tensor) -> torch.Tensor:
    if _gpu(gu):
        out = torch.empty(gu.shape[:-1] + (gu.shape[-1] // 2,), dtype=gu.dtype, device=gu.device)
        ext().silu_mul(out, gu)
        return out
    return ref.silu_mul(gu)


# ----------------------------------------------------------------------------- attention
def rope_and_cache(qkv: torch.Tensor, num_heads: int, num_kv_heads: int, head_dim: int,
                   positions: torch.Tensor, cos_sin: torch.Tensor, kv_layer: torch.Tensor,
                   slot_mapping: torch.Tensor, q_norm_w=None, k_norm_w=None, eps: float = 1e-6,
                   k_scale: float = 1.0, v_scale: float = 1.0):
    """qkv [T, (Hq+2Hkv)*D] (fused projection output).  Applies optional q/k head RMSNorm and RoPE,
    writes K/V into the paged cache (bf16, or fp8 e4m3fn storing x / scale), returns q [T, Hq, D]."""
    T = qkv.shape[0]
    qs, ks = num_heads * head_dim, num_kv_heads * head_dim
    if _gpu(qkv):
        q = torch.empty(T, num_heads, head_dim, dtype=qkv.dtype, device=qkv.device)
        ext().rope_and_cache(q, qkv, positions, cos_sin, kv_layer, slot_mapping,
                             q_norm_w, k_norm_w, num_heads, num_kv_heads, head_dim, eps, k_scale, v_scale)
        return q
    q = qkv[:, :qs].reshape(T, num_heads, head_dim)
    k = qkv[:, qs:qs + ks].reshape(T, num_kv_heads, head_dim)
    v = qkv[:, qs + ks:].reshape(T, num_kv_heads, head_dim)
    return ref.rope_and_cache(q, k, v, positions, cos_sin, kv_layer, slot_mapping, q_norm_w, k_norm_w, eps,
                              k_scale, v_scale)


def qkv_uses_slabs(h: torch.Tensor, w: torch.Tensor) -> bool:
    """Whether linear_rope_and_cache takes its split-K slab path for this qkv projection (then the rope
    kernel reads the unreduced slabs and writes q itself)."""
    if not (_gpu(h) and h.dim() == 2 and 0 < h.shape[0] <= _decode_max_m()):
        return False
    from .decode_gemm import TABLE
    cfg = TABLE.lookup(h.shape[0], w.shape[0], w.shape[1], 0)
    return cfg is not None and TABLE.splitk(cfg) > 1


def linear_rope_and_cache(h: torch.Tensor, w: torch.Tensor, num_heads: int, num_kv_heads: int, head_dim: int,
                          positions: torch.Tensor, cos_sin: torch.Tensor, kv_layer: torch.Tensor,
                          slot_mapping: torch.Tensor, q_norm_w=None, k_norm_w=None, eps: float = 1e-6,
                          k_scale: float = 1.0, v_scale: float = 1.0):
    """qkv projection + rope_and_cache.  When the decode table runs the projection split-K, its fp32
    slabs feed the rope / cache-write kernel directly (no reduce kernel, no bf16 qkv round trip)."""
    if _gpu(h) and h.dim() == 2 and 0 < h.shape[0] <= _decode_max_m() and head_dim in (64, 128):
        from .decode_gemm import TABLE
        M, N = h.shape[0], w.shape[0]
        cfg = TABLE.lookup(M, N, w.shape[1], 0)
        if cfg is not None and TABLE.splitk(cfg) > 1:
            dummy = torch.empty(M, N, dtype=h.dtype, device=h.device)  # not written when the reduce is skipped
            if TABLE.run(dummy, h, w, cfg, 0, reduce=False):
                q = torch.empty(M, num_heads, head_dim, dtype=h.dtype, device=h.device)
                if ext().splitk_rope_and_cache(q, TABLE.part, TABLE.splitk(cfg), M, positions, cos_sin, kv_layer,
                                               slot_mapping, q_norm_w, k_norm_w, num_heads, num_kv_heads, head_dim,
                                               eps, k_scale, v_scale):
                    return q
                TABLE.run(dummy, h, w, cfg, 0)  # kernel shape not covered: reduce and take the plain path
                return rope_and_cache(dummy, num_heads, num_kv_heads, head_dim, positions, cos_sin, kv_layer,
                                      slot_mapping, q_norm_w, k_norm_w, eps, k_scale, v_scale)
    return rope_and_cache(linear(h, w), num_heads, num_kv_heads, head_dim, positions, cos_sin, kv_layer, slot_mapping,
                          q_norm_w, k_norm_w, eps, k_scale, v_scale)


_ROPE_SPLIT = os.environ.get("MXS_ROPE_SPLIT", "1") == "1"  # 0: one launch for mixed steps (A/B)


def rope_kv_into_cache(qkv: torch.Tensor, num_heads: int, num_kv_heads: int, head_dim: int,
                       positions: torch.Tensor, cos_sin: torch.Tensor, kv_layer: torch.Tensor,
                       slot_mapping: torch.Tensor, k_scale: float = 1.0, v_scale: float = 1.0,
                       num_decodes: int = 0) -> torch.Tensor:
    """rope_and_cache without the q write (GPU): RoPE on k, K / V into the paged cache; returns the
    un-rotated q as a row-strided view of qkv, for the attention ops' `rope=` argument.
    num_decodes: a mixed step's leading decode rows (one token per sequence, scattered slots) go to
    the one-token-per-workgroup kernel, the prefill rows to the 16-token tile kernel: a tile of 16
    decode rows is 16 runs of one token, i.e. 8k two-byte V stores on one workgroup, the slowest
    tile of the launch."""
    T = qkv.shape[0]
    parts = [(0, T)]
    if 0 < num_decodes < T and T - num_decodes >= 512 and _ROPE_SPLIT:
        parts = [(0, num_decodes), (num_decodes, T)]
    for a, b in parts:
        ext().rope_and_cache(None, qkv[a:b], positions[a:b], cos_sin, kv_layer, slot_mapping[a:b], None, None,
                             num_heads, num_kv_heads, head_dim, 1e-6, k_scale, v_scale)
    return qkv[:, :num_heads * head_dim].view(T, num_heads, head_dim)


def paged_attention_decode(q: torch.Tensor, kv_layer: torch.Tensor, block_tables: torch.Tensor,
                           seq_lens: torch.Tensor, scale: float, max_seq_len: int,
                           out: Optional[torch.Tensor] = None, k_scale: float = 1.0,
                           v_scale: float = 1.0, impl: Optional[int] = None, rope: Optional[tuple] = None) -> torch.Tensor:
    """One query token per sequence.  q [B, Hq, D] -> [B, Hq, D] (written into `out` if given).
    impl: 0 auto (MFMA kernel from G = 4 query heads per kv head), 1 VALU dot2, 2 MFMA;
    MXS_DECODE_ATTN overrides the default.  rope = (positions [B], cos_sin): q is un-rotated (a
    strided view of the qkv rows) and the kernel applies RoPE while loading it."""
    if _gpu(q):
        out = torch.empty(q.shape, dtype=q.dtype, device=q.device) if out is None else out
        rp, cs = rope if rope is not None else (None, None)
        ext().paged_attention_decode(out, q, kv_layer, block_tables, seq_lens, scale, max_seq_len, k_scale, v_scale,
                                     _DECODE_IMPL if impl is None else impl, rp, cs)
        return out
    if rope is not None:
        q = ref.apply_rope(q, rope[0], rope[1])
    return ref.paged_attention_decode(q, kv_layer, block_tables, seq_lens, scale, k_scale, v_scale)


def paged_attention_prefill(q: torch.Tensor, kv_layer: torch.Tensor, block_tables: torch.Tensor,
                            query_start_loc: torch.Tensor, seq_lens: torch.Tensor, scale: float,
                            max_query_len: int, out: Optional[torch.Tensor] = None,
                            version: int = 0, k_scale: float = 1.0, v_scale: float = 1.0,
                            rope: Optional[tuple] = None) -> torch.Tensor:
    """Causal varlen attention of prefill chunks against the paged cache (prefix included).
    version: 0 = default (v3, LDS-shared K/V tiles; MXS_PREFILL_KERNEL=2 selects v2), 2 or 3.
    rope: as for paged_attention_decode (v3)."""
    if _gpu(q):
        out = torch.empty(q.shape, dtype=q.dtype, device=q.device) if out is None else out
        rp, cs = rope if rope is not None else (None, None)
        ext().paged_attention_prefill(out, q, kv_layer, block_tables, query_start_loc, seq_lens,
                                      scale, max_query_len, version or _PREFILL_VERSION, k_scale, v_scale, rp, cs)
        return out
    if rope is not None:
        q = ref.apply_rope(q, rope[0], rope[1])
    return ref.paged_attention(q, kv_layer, block_tables, query_start_loc, seq_lens, scale, k_scale, v_scale)


# ----------------------------------------------------------------------------- sampling
def sample(logits: torch.Tensor, temperature: torch.Tensor, top_p: torch.Tensor,
           top_k: torch.Tensor, seeds: torch.Tensor, steps: torch.Tensor) -> torch.Tensor:
    if _gpu(logits):
        out = torch.empty(logits.shape[0], dtype=torch.int64, device=logits.device)
        ext().sample(out, logits, temperature, top_p, top_k, seeds, steps)
        return out
    return ref.sample(logits, temperature, top_p, top_k, seeds, steps)


def apply_penalties(logits, hist, srows, hlen, plen, rep, freq, pres, counts=None) -> torch.Tensor:
    """In place on logits [B, V]: repetition (prompt + output), frequency / presence (output)
    penalties from the device token history; `counts` is a [>= B, V] int32 scratch."""
    if _gpu(logits):
        if counts is None:
            counts = torch.empty(logits.shape[0], logits.shape[1], dtype=torch.int32, device=logits.device)
        ext().apply_penalties(logits, hist, srows, hlen, plen, rep, freq, pres, counts)
        return logits
    return ref.apply_penalties(logits, hist, srows, hlen, plen, rep, freq, pres)


def logprobs(logits: torch.Tensor, rows: torch.Tensor, tokens: torch.Tensor, k: int):
    """(token log-prob [n], top ids [n, k], top log-probs [n, k]) for logits rows `rows`."""
    if _gpu(logits):
        n = rows.shape[0]
        tok_lp = torch.empty(n, dtype=torch.float32, device=logits.device)
        top_ids = torch.empty(n, k, dtype=torch.int64, device=logits.device)
        top_lp = torch.empty(n, k, dtype=torch.float32, device=logits.device)
        ext().logprobs(tok_lp, top_ids, top_lp, logits, rows, tokens)
        return tok_lp, top_ids, top_lp
    return ref.logprobs(logits, rows, tokens, k)


# ----------------------------------------------------------------------------- MoE
def moe_topk_softmax(router_logits: torch.Tensor, k: int):
    if _gpu(router_logits):
        T, E = router_logits.shape
        w = torch.empty(T, k, dtype=torch.float32, device=router_logits.device)
        ids = torch.empty(T, k, dtype=torch.int32, device=router_logits.device)
        ext().moe_topk_softmax(w, ids, router_logits)
        return w, ids
    return ref.moe_topk_softmax(router_logits, k)


def moe_experts(x, w13, w2, topk_w, topk_ids, expert_offset: int = 0):
    if _gpu(x):
        from . import moe as _moe
        return _moe.fused_experts(x, w13, w2, topk_w, topk_ids, expert_offset)
    return ref.moe_experts(x, w13, w2, topk_w, topk_ids, expert_offset)
