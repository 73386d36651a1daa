"""hipBLASLt with a measured solution for the prefill projections that stay on the library.

hipBLASLt ships ~230 gfx950 solutions for the bf16 TN GEMM of a linear layer; torch runs the one its
heuristic ranks first, which is not always the fastest at the engine's row counts (a 4,000-token
prompt plus the decode rows: 4-7 k rows).  A start-up tuner (model_runner._tune_gemms, after the
M-plan tuner and before the gemm_pf tuner, which then compares against this path) screens every
solution that supports the shape at each row bucket, re-times the best few against the path it
would replace (ops.linear's route, or addmm_ into the residual stream for o / down) at the bucket's
top and middle row counts, and keeps a solution only where it wins at both by WIN_MARGIN.
csrc/kernels/hblt.cpp runs it (descriptors cached per shape, the solution re-checked per shape).

Solution indices belong to one hipBLASLt build: each entry stores the solution's kernel name, and a
table entry whose index names another kernel in the loaded library is re-measured.
MXS_HBLT=auto (default: the packaged / MXS_TUNED_DIR table only -- a shape it does not hold stays on
torch's call, so start-up stays fast and every process runs the same kernels) | tune (also measure
the shapes the table lacks; with MXS_TUNED_SAVE=1 they are written back) | off.  Choices persist in
mxserve/ops/tuned/prefill_hblt_<arch>_<cus>cu.json.
"""
from __future__ import annotations

import bisect
import os
from typing import Optional

import torch

MODE = os.environ.get("MXS_HBLT", "auto")
WIN_MARGIN = 0.98
SCREEN_KEEP = 6
ROUNDS = 3


class HbltTable:
    """(N, K, resid) -> sorted [(M bucket, solution index | None)]; a row count takes the smallest
    bucket >= M (past the last, the last)."""

    def __init__(self):
        self.entries: dict = {}
        self.report: list = []

    def lookup(self, M: int, N: int, K: int, resid: bool) -> Optional[int]:
        if MODE not in ("auto", "tune") or M <= 256:
            return None
        ent = self.entries.get((N, K, bool(resid)))
        if not ent:
            return None
        i = bisect.bisect_left(ent, (M,))
        return ent[min(i, len(ent) - 1)][1]


TABLE = HbltTable()
# choices measured in this process (not in the packaged table): a later engine start in the same
# process reuses them, so its kernels -- and bf16 roundings -- match the first engine's
_MEASURED: dict = {}


def linear(x: torch.Tensor, w: torch.Tensor) -> Optional[torch.Tensor]:
    """x @ w.T with the tuned solution of this bucket; None when there is none (the caller goes on)."""
    sol = TABLE.lookup(x.shape[0], w.shape[0], w.shape[1], False)
    if sol is None:
        return None
    from .. import ops
    return ops.hblt_mm(x, w, sol)


def addmm_(r: torch.Tensor, x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """r += x @ w.T in place: the tuned solution with beta = 1, else torch's addmm_."""
    sol = TABLE.lookup(x.shape[0], w.shape[0], w.shape[1], True)
    if sol is not None:
        from .. import ops
        if ops.hblt_mm(x, w, sol, out=r, resid=r) is not None:
            return r
    return r.addmm_(x, w.t())


def _points(lo: int, hi: int) -> list:
    """Row counts a bucket (lo, hi] is measured at: its top and its middle."""
    return sorted({hi, max(lo + 1, (lo + hi) // 2)})


def tune(weights: dict, resid_names: set, max_rows: int, device, dtype=torch.bfloat16) -> list:
    """weights: {name: w [N, K]}; resid_names: projections that also run as r += x W^T (o / down of the
    fused prefill chain).  Fills TABLE; returns report rows."""
    if MODE not in ("auto", "tune"):
        return []
    from .. import ops
    from . import prefill_pf
    from .prefill_pf import _time, buckets_for
    from .tuned import TunedStore, device_tag, median
    store = TunedStore("prefill_hblt", device_tag(device))
    rows = []
    saved_pf = prefill_pf.MODE
    for name, w in weights.items():
        N, K = w.shape
        for resid in ((False, True) if name in resid_names else (False,)):
            TABLE.entries.pop((N, K, resid), None)  # the baseline must not route through this table
            ent, lo = [], 256
            for Mb in buckets_for(max_rows):
                key = f"{N}x{K}:{int(resid)}@{Mb}"
                pts = _points(lo, Mb)
                xs: dict = {}
                rs: dict = {}

                def base(M):
                    if resid:
                        return rs[M].addmm_(xs[M], w.t())
                    prefill_pf.MODE = "off"  # the path hblt replaces: hipBLASLt's own pick or an M plan
                    try:
                        return ops.linear(xs[M], w)
                    finally:
                        prefill_pf.MODE = saved_pf

                def run(sol, M):
                    return ops.hblt_mm(xs[M], w, sol, out=rs[M] if resid else None, resid=rs[M] if resid else None)

                st = store.get(key) or _MEASURED.get((store.tag, key))
                if st is not None and st.get("sol") is not None and \
                        ops.ext().hblt_kernel_name(int(st["sol"])) != st.get("kernel"):
                    st = None  # another hipBLASLt build: its index names another kernel
                if st is not None:
                    sol, t_best, t_base, source = st.get("sol"), st.get("us"), st.get("base_us"), "table"
                elif MODE != "tune":  # not in the table: torch's call (measuring is opt-in)
                    ent.append((Mb, None))
                    lo = Mb
                    continue
                xs.update({M: (torch.rand(M, K, device=device) * 2 - 1).to(dtype) for M in pts})
                if resid:
                    rs.update({M: (torch.rand(M, N, device=device) * 2 - 1).to(dtype) for M in pts})
                if st is None:  # MXS_HBLT=tune and not in the table: measure
                    source = "measured"
                    top = pts[-1]
                    screen = {}
                    for c in ops.hblt_candidates(top, N, K, resid):
                        if run(c, top) is None or any(run(c, M) is None for M in pts):
                            continue
                        screen[c] = _time(lambda c=c: run(c, top), 3)
                    keep = sorted(screen, key=screen.get)[:SCREEN_KEEP]
                    tb = {M: [] for M in pts}
                    tc = {(c, M): [] for c in keep for M in pts}
                    for _ in range(ROUNDS):
                        for M in pts:
                            tb[M].append(_time(lambda M=M: base(M)))
                            for c in keep:
                                tc[(c, M)].append(_time(lambda c=c, M=M: run(c, M)))
                    base_t = {M: median(tb[M]) for M in pts}
                    t_base = sum(base_t.values())
                    sol, t_best = None, t_base
                    for c in keep:
                        t = {M: median(tc[(c, M)]) for M in pts}
                        if all(t[M] < base_t[M] for M in pts) and sum(t.values()) < t_base * WIN_MARGIN \
                                and sum(t.values()) < t_best:
                            sol, t_best = c, sum(t.values())
                if sol is not None:  # correctness against the path it replaces, at the bucket's top
                    M = pts[-1]
                    if resid:
                        r0 = rs[M].clone()
                        want = r0.float() + (xs[M].float() @ w.float().t())
                        got = ops.hblt_mm(xs[M], w, sol, out=None, resid=r0)
                    else:
                        want = base(M).float()
                        got = ops.hblt_mm(xs[M], w, sol)
                    if got is None or not (got.float() - want).abs().max().item() <= 0.02 * max(1.0, want.abs().max().item()):
                        sol, t_best = None, t_base
                if source == "measured":
                    ent_d = {"sol": sol, "kernel": ops.ext().hblt_kernel_name(int(sol)) if sol is not None else None,
                             "us": t_best and round(t_best, 2), "base_us": round(t_base, 2), "points": pts}
                    store.put(key, ent_d)
                    _MEASURED[(store.tag, key)] = ent_d
                ent.append((Mb, sol))
                rows.append({"proj": name, "M": Mb, "N": N, "K": K, "resid": resid, "base_us": t_base and round(t_base, 2),
                             "chosen": "default" if sol is None else f"sol{sol}", "us": t_best and round(t_best, 2),
                             "source": source})
                lo = Mb
            TABLE.entries[(N, K, resid)] = ent
    TABLE.report = rows
    store.save()
    return rows
