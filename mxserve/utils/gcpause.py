"""Python garbage-collector pauses on the engine thread.

A serving process holds a large, long-lived heap after start-up (torch, the model runner's graph
pools, tokenizer tables): a full (generation-2) collection walks every tracked object in it and,
at the headline operating point, stalled the step loop for ~110 ms at a time with the GPU idle
(profiles/r3/s3/busy_q46.json: two 114 ms gaps between steps in a 6 s window, 4 % of the wall).
`freeze_heap()` moves everything alive at the end of engine start-up into the permanent
generation (gc.freeze), so later collections only walk what the serving loop allocates, and raises
the young-generation threshold so the per-token garbage (StepOutput, small lists) is collected in
fewer, equally cheap passes.  `PauseStats` records every collection's duration through
gc.callbacks, so a benchmark can report the worst pause it saw.

MXS_GC_FREEZE=0 leaves the collector untouched.
"""
from __future__ import annotations

import gc
import os
import time
from typing import Optional

_FROZEN = False


def freeze_heap(gen0_threshold: int = 20000) -> bool:
    """Collect once, freeze the survivors, widen gen 0.  Idempotent per process; returns whether the
    heap was frozen by this call."""
    global _FROZEN
    if os.environ.get("MXS_GC_FREEZE", "1") != "1" or not hasattr(gc, "freeze"):
        return False
    gc.collect()
    gc.freeze()
    t0, t1, t2 = gc.get_threshold()
    if t0 < gen0_threshold:
        gc.set_threshold(gen0_threshold, t1, t2)
    first = not _FROZEN
    _FROZEN = True
    return first


def unfreeze_heap() -> None:
    """Return frozen objects to the collector (an engine being torn down was frozen with the rest of
    the start-up heap; without this its reference cycles, and the device memory they hold, would
    never be freed)."""
    global _FROZEN
    if _FROZEN and hasattr(gc, "unfreeze"):
        gc.unfreeze()
        _FROZEN = False


class PauseStats:
    """Durations of the collector's passes while installed (gc.callbacks), per generation."""

    def __init__(self):
        self.n = [0, 0, 0]
        self.total_s = [0.0, 0.0, 0.0]
        self.max_s = [0.0, 0.0, 0.0]
        self._t: Optional[float] = None
        self._installed = False

    def _cb(self, phase: str, info: dict) -> None:
        if phase == "start":
            self._t = time.perf_counter()
        elif self._t is not None:
            g = int(info.get("generation", 0))
            d = time.perf_counter() - self._t
            self._t = None
            self.n[g] += 1
            self.total_s[g] += d
            self.max_s[g] = max(self.max_s[g], d)

    def install(self) -> "PauseStats":
        if not self._installed:
            gc.callbacks.append(self._cb)
            self._installed = True
        return self

    def remove(self) -> None:
        if self._installed:
            gc.callbacks.remove(self._cb)
            self._installed = False

    def summary(self) -> dict:
        return {"frozen": _FROZEN, "collections": list(self.n),
                "total_ms": [round(1e3 * s, 2) for s in self.total_s],
                "max_ms": [round(1e3 * s, 2) for s in self.max_s]}
