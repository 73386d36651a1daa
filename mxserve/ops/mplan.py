"""Prefill M plans: how to run a prefill / mixed-step projection GEMM of M rows on hipBLASLt.

hipBLASLt picks its kernel by heuristic, and the choice has cliffs in the row count: on MI355X the
Llama-3.2-1B gate_up takes 189 us at 4096 rows and 247 us at 4224-4352 (a mixed step with one
4000-token prompt and ~270 decode rows), down 171 us at 8192 and 396 us at 8320, and F.linear and
mm(out=) sometimes run different kernels for the same shape (profiles/r3/s3/hipblaslt_m_sweep.jsonl).
A plan for an M bucket (128 rows) is a list of (rows, form) segments, form "lin" (F.linear) or "mm"
(torch.mm into a slice of the output); a split runs a sweet-spot block and the remainder as two
calls into one output tensor.

The table per device lives in ops/tuned/prefill_mplan_<arch>_<cus>cu.json (the packaged MI355X one
was built from the 128-row sweep above).  `tune()` fills in shapes the table lacks at engine
start-up from a coarser sweep (every `grid` rows up to the step's token budget, both call forms,
median of 3 timings each) and keeps a plan only where it predicts >= 4 % over one F.linear;
MXS_TUNED_SAVE=1 writes the grown table back (ops/tuned.py conventions).  ops.linear consults it.
"""
from __future__ import annotations

import json
import logging
import os
import time
from typing import Optional

import torch

log = logging.getLogger(__name__)

LAUNCH_US = 3.0  # a second call in a split
COPY_BPS = 5e12  # a "lin" segment inside a split writes a fresh tensor that is copied into place
MIN_GAIN = 0.96  # a plan must predict <= 96 % of one F.linear


def plans_from_times(times: dict, N: int) -> dict:
    """times: {M: (F.linear us, mm(out=) us)} on a row grid -> {str(M): {"plan", "us", "linear_us"}}
    for the buckets where a single other form or a two-segment split beats F.linear by the margin."""
    grid = sorted(times)
    out = {}
    for M in grid:
        lin, mm = times[M]
        best = (lin, [[M, "lin"]]) if lin <= mm else (mm, [[M, "mm"]])
        for a in grid:
            if a >= M:
                break
            b = M - a
            if b not in times:
                continue
            cost, segs = LAUNCH_US, []
            for rows in (a, b):
                tl, tm = times[rows]
                copy = rows * N * 4 / COPY_BPS * 1e6  # us: read + write of the segment's bf16 output
                if tm <= tl + copy:
                    cost += tm
                    segs.append([rows, "mm"])
                else:
                    cost += tl + copy
                    segs.append([rows, "lin"])
            if cost < best[0]:
                best = (cost, segs)
        if best[0] < lin * MIN_GAIN:
            out[str(M)] = {"plan": best[1], "us": round(best[0], 1), "linear_us": round(lin, 1)}
    return out


def _time_us(fn, iters: int = 6) -> float:
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


def sweep(w: torch.Tensor, max_m: int, grid: int = 256, rounds: int = 3) -> dict:
    """{M: (F.linear us, mm(out=) us)} for M = grid, 2 grid, ... <= max_m (median of `rounds`)."""
    from .tuned import median
    N, K = w.shape
    x = torch.randn(max_m, K, device=w.device, dtype=w.dtype)
    y = torch.empty(max_m, N, device=w.device, dtype=w.dtype)
    out = {}
    for M in range(grid, max_m + 1, grid):
        xs, ys = x[:M], y[:M]
        lin, mm = [], []
        for _ in range(rounds):
            lin.append(_time_us(lambda: torch.nn.functional.linear(xs, w)))
            mm.append(_time_us(lambda: torch.mm(xs, w.t(), out=ys)))
        out[M] = (median(lin), median(mm))
    return out


def table_path(device, write: bool = False) -> str:
    from .tuned import PKG_DIR, device_tag
    name = f"prefill_mplan_{device_tag(device)}.json"
    d = os.environ.get("MXS_TUNED_DIR")
    if d and (write or os.path.exists(os.path.join(d, name))):
        return os.path.join(d, name)
    return os.path.join(PKG_DIR, name)


def load(device) -> dict:
    try:
        with open(table_path(device)) as f:
            return json.load(f).get("entries", {})
    except (OSError, ValueError):
        return {}


def tune(weights: dict, max_m: int, device, grid: int = 256) -> dict:
    """Measure plans for the prefill projection shapes (name -> [N, K] weight) that the device's table
    lacks; returns {"shapes_tuned": [...], "tune_s": ...}.  The ops-level table is updated in place."""
    from . import _MPLAN
    if os.environ.get("MXS_MPLAN", "1") != "1" or os.environ.get("MXS_MPLAN_TUNE", "1") != "1":
        return {}
    tab = _MPLAN.get(device)
    if tab is None:
        tab = _MPLAN[device] = load(device)
    t0 = time.time()
    done = []
    for name, w in weights.items():
        N, K = w.shape
        key = f"{N}x{K}"
        if key in tab or max_m < 2 * grid:
            continue
        with torch.inference_mode():
            times = sweep(w, max_m, grid)
        tab[key] = plans_from_times(times, N)
        done.append(name)
    rep = {"shapes_tuned": done, "tune_s": round(time.time() - t0, 2)}
    if done and os.environ.get("MXS_TUNED_SAVE") == "1":
        from .tuned import device_tag
        path = table_path(device, write=True)
        os.makedirs(os.path.dirname(path), exist_ok=True)
        with open(path, "w") as f:
            json.dump({"kind": "prefill_mplan", "device": device_tag(device), "entries": tab}, f, indent=0)
            f.write("\n")
    if done:
        log.info("prefill M plans tuned for %s in %.1fs", done, rep["tune_s"])
    return rep
