"""Decode projection GEMMs on the hand-written MFMA kernel (csrc/kernels/gemm_decode.hip), chosen per
(batch bucket, projection) by measurement.

When the decode graphs are captured, ModelRunner calls `tune()` with the model's projection shapes
(qkv, o, gate_up with SiLU*mul fused, down, lm_head) and the graph batch buckets.  For every pair it
times hipBLASLt (+ the separate SiLU*mul kernel for gate_up) and a set of kernel configurations
(wave tile MF x NF fragments, wave layout, split-K), each as 20 calls replayed from one hipGraph
(no launch gaps, the way the decode graphs run them), checks the winner against hipBLASLt's output
and records it.  `linear()` / `gate_up_silu()` then use the table; anything not tuned, or where
hipBLASLt won, stays on hipBLASLt.  MXS_DECODE_GEMM=off disables the kernel, =force uses a default
configuration without timing (tests).
"""
from __future__ import annotations

import bisect
import json
import logging
import os
import time
from typing import Optional

import torch

log = logging.getLogger(__name__)

MAX_M = 256
# buckets the capture-time tuner measures: above this the register-staged kernel measured 1.3-2.5x
# behind hipBLASLt for every projection (profiles/r2_decode_gemm_probe_vs_hipblaslt.jsonl), so the
# engine does not spend startup time timing them
MAX_TUNE_M = int(os.environ.get("MXS_DECODE_GEMM_TUNE_MAX_M", "64"))
MODE = os.environ.get("MXS_DECODE_GEMM", "auto")  # auto | off | force


def _mf(M: int) -> int:
    return 1 if M <= 16 else (2 if M <= 32 else 4)


def unroll(mf: int, nf: int) -> int:
    """k-steps per load group (csrc/kernels/gemm_decode.hip decode_gemm_unroll)."""
    return 8 if mf + nf <= 3 else (4 if mf + nf <= 6 else 2)


def candidates(M: int, N: int, K: int, epi: int, all_mf: bool = False, lds: bool = True) -> list[tuple]:
    """(mf, nf, wm, splitk, lu) configurations that tile the shape (wave row tile MF x 16 sized to M
    unless all_mf: then every MF, i.e. more row tiles re-reading the weights from L2).  lu = 0: the
    register kernel (wm waves over M); lu = 2 / 4: the LDS form (X tile shared by the workgroup's 4
    waves through LDS, lu k-steps per group)."""
    out = []
    for mf in ((1, 2, 4) if all_mf else (_mf(M),)):
        out += _candidates_mf(M, N, K, epi, mf)
        if lds and mf > 1:  # one 16-row tile: the X fragment is as small as one W fragment
            out += _candidates_lds(N, K, epi, mf)
    return out


def _candidates_lds(N: int, K: int, epi: int, mf: int) -> list[tuple]:
    out = []
    for nf in (2, 4):
        nh = nf // 2 if epi else nf
        if (N // 2 if epi else N) % (4 * nh * 16):
            continue
        for lu in (2, 4):
            for sk in (1, 2, 4, 8):
                if K % (32 * lu * sk) == 0:
                    out.append((mf, nf, 1, sk, lu))
    return out


def _candidates_mf(M: int, N: int, K: int, epi: int, mf: int) -> list[tuple]:
    out = []
    for wm in (1, 2, 4):
        if wm > 1 and (wm // 2) * mf * 16 >= M:  # waves with no rows at all
            continue
        wn = 4 // wm
        for nf in (2, 4):
            nh = nf // 2 if epi else nf
            outN = N // 2 if epi else N
            if outN % (wn * nh * 16):
                continue
            for sk in (1, 2, 4, 8):
                if K % (32 * unroll(mf, nf) * sk):
                    continue
                out.append((mf, nf, wm, sk, 0))
    return out


class DecodeGemmTable:
    def __init__(self):
        self.entries: dict[tuple, list] = {}  # (N, K, epi) -> sorted [(M bucket, cfg or None)]
        self.part: Optional[torch.Tensor] = None  # fp32 split-K workspace (stable for graphs)
        self.report: list = []

    def lookup(self, M: int, N: int, K: int, epi: int) -> Optional[tuple]:
        if MODE == "off" or M > MAX_M:
            return None
        if MODE == "force":
            c = candidates(M, N, K, epi)
            return next((x for x in c if x[3] == 1), c[0] if c else None)
        ent = self.entries.get((N, K, epi))
        if not ent:
            return None
        i = bisect.bisect_left(ent, (M,))
        if i == len(ent):
            return None
        return ent[i][1]

    def run(self, out: torch.Tensor, x: torch.Tensor, w: torch.Tensor, cfg: tuple, epi: int) -> bool:
        from . import ext
        mf, nf, wm, sk = cfg[:4]
        lu = cfg[4] if len(cfg) > 4 else 0
        part = None
        if sk > 1:
            need = sk * x.shape[0] * w.shape[0]
            if self.part is None or self.part.numel() < need:
                if torch.cuda.is_current_stream_capturing():
                    return False  # never allocate inside a capture (tune() sizes it beforehand)
                self.part = torch.empty(need, dtype=torch.float32, device=x.device)
            part = self.part
        return bool(ext().decode_gemm(out, x, w, part, mf, nf, wm, sk, epi, lu))


TABLE = DecodeGemmTable()


def _graph_time(fn, iters: int = 20) -> float:
    """Microseconds per call of `fn`, from `iters` calls captured in one hipGraph."""
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
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    del g
    return e0.elapsed_time(e1) * 1e3 / iters


def tune(shapes: dict, buckets: list, device, dtype=torch.bfloat16) -> list:
    """shapes: {name: (weight tensor [N, K], epi)}.  Fills TABLE; returns the report rows."""
    if MODE != "auto":
        return []
    from . import ext, silu_mul
    t0 = time.time()
    bks = sorted(b for b in buckets if b <= min(MAX_M, MAX_TUNE_M))
    if not bks:
        return []
    # workspace for the largest split-K any candidate may pick
    need = max(8 * max(bks) * w.shape[0] for w, _ in shapes.values())
    TABLE.part = torch.empty(need, dtype=torch.float32, device=device)
    rows = []
    for name, (w, epi) in shapes.items():
        N, K = w.shape
        ent = []
        for M in bks:
            x = (torch.randn(M, K, device=device) * 0.5).to(dtype)
            outN = N // 2 if epi else N
            ref_out = silu_mul(torch.nn.functional.linear(x, w)) if epi else torch.nn.functional.linear(x, w)
            if epi:
                t_lib = _graph_time(lambda: silu_mul(torch.nn.functional.linear(x, w)))
            else:
                t_lib = _graph_time(lambda: torch.nn.functional.linear(x, w))
            best, best_t = None, t_lib
            out = torch.empty(M, outN, dtype=dtype, device=device)
            for cfg in candidates(M, N, K, epi):
                if not TABLE.run(out, x, w, cfg, epi):
                    continue
                t = _graph_time(lambda: TABLE.run(out, x, w, cfg, epi))
                if t < best_t * 0.97:  # a clear win only
                    best, best_t = cfg, t
            if best is not None:  # correctness gate: the winner must match hipBLASLt's result
                TABLE.run(out, x, w, best, epi)
                err = (out.float() - ref_out.float()).abs().max().item()
                tol = 0.02 * max(1.0, ref_out.float().abs().max().item())
                if not err <= tol:
                    log.warning("decode GEMM %s M=%d cfg %s mismatches hipBLASLt (%.3g); not used", name, M, best, err)
                    best, best_t = None, t_lib
            ent.append((M, best))
            rows.append({"proj": name, "M": M, "N": N, "K": K, "epi": epi, "hipblaslt_us": round(t_lib, 2),
                         "chosen": "hipblaslt" if best is None else "mfma", "cfg": best, "us": round(best_t, 2)})
        TABLE.entries[(N, K, epi)] = ent
    TABLE.report = rows
    won = sum(r["chosen"] == "mfma" for r in rows)
    log.info("decode GEMM tuning: MFMA kernel chosen for %d of %d (bucket, projection) pairs in %.1fs", won,
             len(rows), time.time() - t0)
    path = os.environ.get("MXS_DECODE_GEMM_REPORT")
    if path:
        with open(path, "w") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")
    return rows


class PrefillGemmTable:
    """Prefill-sized GEMMs (256 < M <= PREFILL_MAX_M) on the tile kernel of gemm_prefill.hip where
    the startup measurement found it faster than hipBLASLt: (N, K) -> sorted [(M bucket, cfg|None)].
    Above PREFILL_MAX_M the library's 256 x 256 tiles fill the chip and win
    (profiles/r2_prefill_gemm_probe_v1.jsonl)."""

    def __init__(self):
        self.entries: dict = {}
        self.report: list = []

    def lookup(self, M: int, N: int, K: int):
        if MODE == "off" or M > PREFILL_MAX_M:
            return None
        ent = self.entries.get((N, K))
        if not ent:
            return None
        i = bisect.bisect_left(ent, (M,))
        return ent[i][1] if i < len(ent) else None


PREFILL_MAX_M = int(os.environ.get("MXS_PREFILL_GEMM_MAX_M", "768"))
PREFILL_TABLE = PrefillGemmTable()


def _event_time(fn, iters: int = 10) -> float:
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


def tune_prefill(weights: dict, device, dtype=torch.bfloat16, buckets=(384, 512, 768)) -> list:
    """weights: {name: [N, K] tensor}.  Per M bucket: every tile / split-K configuration of the
    prefill kernel vs hipBLASLt (eager launches, as prefill runs), correctness-gated."""
    if MODE != "auto":
        return []
    from .. import ops
    rows = []
    for name, w in weights.items():
        N, K = w.shape
        ent = []
        for M in sorted(b for b in buckets if 256 < b <= PREFILL_MAX_M):
            x = (torch.randn(M, K, device=device) * 0.5).to(dtype)
            ref = torch.nn.functional.linear(x, w)
            t_lib = _event_time(lambda: torch.nn.functional.linear(x, w))
            best, best_t = None, t_lib
            out = torch.empty(M, N, dtype=dtype, device=device)
            for cfg in ops.prefill_gemm_configs(M, N, K):
                if not ops.prefill_gemm(out, x, w, cfg):
                    continue
                t = _event_time(lambda: ops.prefill_gemm(out, x, w, cfg))
                if t < best_t * 0.97:
                    best, best_t = cfg, t
            if best is not None:
                ops.prefill_gemm(out, x, w, best)
                err = (out.float() - ref.float()).abs().max().item()
                if not err <= 0.02 * max(1.0, ref.float().abs().max().item()):
                    best, best_t = None, t_lib
            ent.append((M, best))
            rows.append({"proj": name, "M": M, "N": N, "K": K, "hipblaslt_us": round(t_lib, 2),
                         "chosen": "hipblaslt" if best is None else "mfma", "cfg": best, "us": round(best_t, 2)})
        PREFILL_TABLE.entries[(N, K)] = ent
    PREFILL_TABLE.report = rows
    return rows
