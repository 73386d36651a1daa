"""Routing of prefill-sized projection GEMMs (M > 256 rows) to the hand-written persistent stream-K
kernel (csrc/kernels/gemm_pf.hip, ops.gemm_pf) instead of hipBLASLt (+ the separate SiLU*mul pass
after gate_up).

A start-up tuner (run with the decode-GEMM tuning at graph capture, model_runner._capture_graphs)
times, per projection and row bucket, gemm_pf at a few minimum stream-K segment lengths against the
path it replaces (ops.linear's hipBLASLt / M-plan route; for gate_up the GEMM plus ops.silu_mul) and
keeps gemm_pf where it is faster.  Choices persist in mxserve/ops/tuned/prefill_pf_<arch>_<cus>cu.json
like the other tables (ops/tuned.py), so every start-up on the same hardware runs the same kernels.

MXS_GEMM_PF=auto (default: the tuned table) | on (gemm_pf for every supported shape, min_iters 16;
tests, probes) | off (never).

Fused prefill chain (models/llama.py _forward_pf, TP = 1 dense models): the RMSNorms run inside
their consumer GEMMs (gemm_pf row scale over the norm-folded qkv / gate_up weights: table codes
3 = plain, 4 = SwiGLU) and the residual adds inside their producers (code 2: gemm_pf epi 2, r += x
W^T in place).  tune_fused() times each against the unfused alternative at the same row buckets
(codes 3 / 4: RMSNorm pass + the routed GEMM; code 2: hipBLASLt addmm_ with beta = 1, or GEMM + add)
and keeps the faster; norm_linear() / resid_linear() run the choice.
"""
from __future__ import annotations

import bisect
import os
from typing import Optional

import torch

MODE = os.environ.get("MXS_GEMM_PF", "auto")
MIN_ITERS = (0, 8, 16, 32)  # 0: data-parallel tiles only (no stream-K)
# (token-tile rows, min_iters) candidates of the plain / SwiGLU / residual forms: the 256-row tile is the
# most efficient per CU, the shorter ones fill the CUs when 256-row tiles leave a partial last round
# (qkv at 6,144 rows: 192-row tiles 1.16x hipBLASLt where 256 reach 0.92x, profiles/r5/prefill_gemm)
CANDIDATES = tuple((256, mi) for mi in MIN_ITERS) + ((224, 0), (224, 16), (192, 0), (192, 32), (160, 0), (160, 32), (128, 0), (128, 8))
WIN_MARGIN = 0.98  # gemm_pf must be this much faster than the path it replaces
ROUNDS = 3


def pf_cfg(cfg) -> tuple:
    """(min_iters, token-tile rows) of a stored gemm_pf choice: an int is min_iters at 256 rows (tables
    of earlier rounds), a pair is [rows, min_iters]."""
    if isinstance(cfg, (list, tuple)):
        return int(cfg[1]), int(cfg[0])
    return int(cfg), 256


def is_pf(cfg) -> bool:
    return isinstance(cfg, int) or (isinstance(cfg, (list, tuple)) and len(cfg) == 2)


def buckets_for(max_rows: int) -> list:
    """Row buckets up to max_rows (a step's largest token count): 512-row steps to 4 k, then 1 k."""
    out, m = [], 512
    while m < max_rows:
        out.append(m)
        m += 512 if m < 4096 else 1024
    out.append(max(max_rows, 512))
    return sorted(set(out))


class PfTable:
    """(N, K, epi) -> sorted [(M bucket, min_iters | None)]; a row count takes its bucket (the
    smallest bucket >= M; past the last, the last)."""

    def __init__(self):
        self.entries: dict = {}
        self.report: list = []

    def lookup(self, M: int, N: int, K: int, epi: int):
        """The gemm_pf choice for this (shape, code) at M rows (pf_cfg() unpacks it), None for the
        unfused path; code 2 may also hold "addmm" (hipBLASLt with beta = 1)."""
        if MODE == "off" or M <= 256 or N % 256 or K % 64:
            return None
        if MODE == "on":
            return 16
        ent = self.entries.get((N, K, epi))
        if not ent:
            return None
        i = bisect.bisect_left(ent, (M,))
        return ent[min(i, len(ent) - 1)][1]


TABLE = PfTable()


def _time(fn, iters: int = 8) -> float:
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


def tune(weights: dict, max_rows: int, device, dtype=torch.bfloat16) -> list:
    """weights: {name: (w [N, K], epi)} (epi 1: gate_up with SiLU*mul).  Fills TABLE; returns report
    rows.  Stored choices are re-checked for correctness, not re-timed."""
    if MODE != "auto":
        return []
    from .. import ops
    from .tuned import TunedStore, device_tag, median
    store = TunedStore("prefill_pf", device_tag(device))
    rows = []
    saved_mode = globals()["MODE"]
    for name, (w, epi) in weights.items():
        N, K = w.shape
        if N % 256 or K % 64:
            continue
        ent = []
        for M in buckets_for(max_rows):
            key = f"{N}x{K}:{epi}@{M}"
            x = (torch.randn(M, K, device=device) * 0.5).to(dtype)

            def base():
                globals()["MODE"] = "off"
                try:
                    y = ops.linear(x, w)
                    return ops.silu_mul(y) if epi == 1 else y
                finally:
                    globals()["MODE"] = saved_mode
            ref = base()
            out = torch.empty(M, N // 2 if epi == 1 else N, dtype=dtype, device=device)
            st = store.get(key)
            if st is not None:
                best, best_t, t_base, source = st.get("cfg"), st.get("us"), st.get("base_us"), "table"
            else:
                source = "measured"
                tb, tc = [], {c: [] for c in CANDIDATES}
                for _ in range(ROUNDS):
                    tb.append(_time(base))
                    for c in CANDIDATES:
                        tc[c].append(_time(lambda: ops.gemm_pf(x, w, epi, out, c[1], trows=c[0])))
                t_base = median(tb)
                best, best_t = None, t_base
                for c in CANDIDATES:
                    t = median(tc[c])
                    if t < t_base * WIN_MARGIN and t < best_t:
                        best, best_t = list(c), t
            if best is not None:
                mi, tr = pf_cfg(best)
                ops.gemm_pf(x, w, epi, out, mi, trows=tr)
                err = (out.float() - ref.float()).abs().max().item()
                if not err <= 0.02 * max(1.0, ref.float().abs().max().item()):
                    best, best_t = None, t_base
            if source == "measured":
                store.put(key, {"cfg": best, "us": best_t and round(best_t, 2), "base_us": round(t_base, 2)})
            ent.append((M, best))
            rows.append({"proj": name, "M": M, "N": N, "K": K, "epi": epi, "base_us": t_base and round(t_base, 2),
                         "chosen": "hipblaslt" if best is None else "gemm_pf/%d/%d" % pf_cfg(best)[::-1],
                         "us": best_t and round(best_t, 2), "source": source})
        TABLE.entries[(N, K, epi)] = ent
    TABLE.report = rows
    store.save()
    return rows


# ----------------------------------------------------------------------------- fused prefill chain
CODE_RESID, CODE_RS, CODE_RS_SWIGLU = 2, 3, 4


def norm_linear(r: torch.Tensor, w: torch.Tensor, wf: Optional[torch.Tensor], norm_w: torch.Tensor, eps: float,
                epi: int) -> torch.Tensor:
    """RMSNorm(r, norm_w) @ w.T (epi 0) or SiLU(. @ gate.T) * (. @ up.T) (epi 1).  gemm_pf with the
    row scale over wf = fold_norm_weight(w, norm_w) where tuned faster, else a norm pass + the
    routed unfused GEMM."""
    from .. import ops
    mi = TABLE.lookup(r.shape[0], w.shape[0], w.shape[1], CODE_RS + epi) if wf is not None else None
    if is_pf(mi):
        out = ops.gemm_pf(r, wf, epi, None, pf_cfg(mi)[0], row_scale=True, eps=eps)
        if out is not None:
            return out
    x = ops.rms_norm(r, norm_w, eps)
    return ops.linear(x, w) if epi == 0 else ops.gate_up_silu(x, w)


def resid_linear(x: torch.Tensor, w: torch.Tensor, r: torch.Tensor) -> torch.Tensor:
    """r += x @ w.T in place (o_proj / down_proj into the residual stream)."""
    from .. import ops
    mi = TABLE.lookup(x.shape[0], w.shape[0], w.shape[1], CODE_RESID)
    if is_pf(mi) and ops.gemm_pf(x, w, 2, r, pf_cfg(mi)[0], resid=r, trows=pf_cfg(mi)[1]) is not None:
        return r
    if mi == "addmm":
        from . import prefill_hblt
        return prefill_hblt.addmm_(r, x, w)  # its tuned solution, else torch's addmm_
    return r.add_(ops.linear(x, w))


def folded_weight_needed(N: int, K: int, code: int, max_rows: int, device) -> bool:
    """Before the KV pool is sized: will the row-scaled form (codes 3 / 4) over a norm-folded copy of
    an [N, K] weight possibly run?  Off -> never; on -> always; auto -> unless the stored table already
    rejects it at every row bucket (then no folded copy is made, and its bytes go to the KV pool)."""
    if MODE == "off" or N % 256 or K % 64:
        return False
    if MODE == "on":
        return True
    from .tuned import TunedStore, device_tag
    store = TunedStore("prefill_pf", device_tag(device))
    for M in buckets_for(max_rows):
        st = store.get(f"{N}x{K}:{code}@{M}")
        if st is None or is_pf(st.get("cfg")):
            return True  # not measured here yet, or gemm_pf kept at this bucket (int or [rows, min_iters])
    return False


def tune_fused(weights: dict, max_rows: int, device, dtype=torch.bfloat16, eps: float = 1e-5) -> list:
    """weights: {name: (w, wf | None, code)} with code 3 / 4 (row-scaled consumer, wf the folded
    weight) or 2 (residual producer).  Adds the codes' entries to TABLE (run after tune(): the
    unfused alternatives route through its choices); returns report rows."""
    if MODE != "auto":
        return []
    from .. import ops
    from . import prefill_hblt
    from .tuned import TunedStore, device_tag, median
    store = TunedStore("prefill_pf", device_tag(device))
    rows = []
    for name, (w, wf, code) in weights.items():
        N, K = w.shape
        if N % 256 or K % 64:
            continue
        epi = code - CODE_RS if code != CODE_RESID else 2
        ent = []
        for M in buckets_for(max_rows):
            key = f"{N}x{K}:{code}@{M}"
            st = store.get(key)
            x = (torch.randn(M, K, device=device) * (2.0 if code != CODE_RESID else 0.5)).to(dtype)
            if st is not None:
                best, best_t, t_base, source = st.get("cfg"), st.get("us"), st.get("base_us"), "table"
            else:
                source = "measured"
                nw = torch.ones(K, device=device, dtype=dtype)
                if code == CODE_RESID:
                    r = torch.randn(M, N, device=device).to(dtype)
                    bases = {None: lambda: r.add_(ops.linear(x, w)), "addmm": lambda: prefill_hblt.addmm_(r, x, w)}
                    cand = {c: (lambda c=c: ops.gemm_pf(x, w, 2, r, c[1], resid=r, trows=c[0])) for c in CANDIDATES}
                else:
                    bases = {None: (lambda: ops.linear(ops.rms_norm(x, nw, eps), w)) if epi == 0 else
                             (lambda: ops.gate_up_silu(ops.rms_norm(x, nw, eps), w))}
                    cand = {(256, mi): (lambda mi=mi: ops.gemm_pf(x, wf, epi, None, mi, row_scale=True, eps=eps))
                            for mi in MIN_ITERS}
                tb = {k: [] for k in bases}
                tc = {k: [] for k in cand}
                for _ in range(ROUNDS):
                    for k, fn in bases.items():
                        tb[k].append(_time(fn))
                    for k, fn in cand.items():
                        tc[k].append(_time(fn))
                bk = min(tb, key=lambda k: median(tb[k]))
                t_base = median(tb[bk])
                best, best_t = bk, t_base
                for c in cand:
                    t = median(tc[c])
                    if t < t_base * WIN_MARGIN and t < best_t:
                        best, best_t = list(c), t
            if is_pf(best):  # correctness of the kept kernel against the unfused path
                bmi, btr = pf_cfg(best)
                if code == CODE_RESID:
                    r0 = torch.randn(M, N, device=device).to(dtype)
                    want = r0.float() + ops.linear(x, w).float()
                    got = ops.gemm_pf(x, w, 2, None, bmi, resid=r0, trows=btr)
                else:
                    want = ops.linear(ops.rms_norm(x, torch.ones(K, device=device, dtype=dtype), eps), w)
                    if epi == 1:
                        want = ops.silu_mul(want)
                    want = want.float()
                    got = ops.gemm_pf(x, w, epi, None, bmi, row_scale=True, eps=eps)
                err = (got.float() - want).abs().max().item()
                if not err <= 0.03 * max(1.0, want.abs().max().item()):
                    best, best_t = None, t_base
            if source == "measured":
                store.put(key, {"cfg": best, "us": best_t and round(best_t, 2), "base_us": round(t_base, 2)})
            ent.append((M, best))
            rows.append({"proj": name, "M": M, "N": N, "K": K, "code": code, "base_us": t_base and round(t_base, 2),
                         "chosen": ("gemm_pf/%d/%d" % pf_cfg(best)[::-1]) if is_pf(best) else (best or "unfused"),
                         "us": best_t and round(best_t, 2), "source": source})
        TABLE.entries[(N, K, code)] = ent
    TABLE.report = TABLE.report + rows
    store.save()
    return rows
