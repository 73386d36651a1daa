"""Request tracing and fault injection.

Tracing: every request gets spans (receive -> tokenize -> route -> first_token -> done) stamped with
its `x-request-id`; finished traces are emitted as one JSON log line (logger `mxserve.trace`) when
MXS_TRACE=1 and kept in a bounded in-memory ring served at /debug/traces.  GPU-side, engine steps are
bracketed with roctx ranges when MXS_ROCTX=1 so rocprofv3 timelines show scheduler steps.

Fault injection (tests only): MXS_FAULT="drop_stream:0.05,fail_prefill:1.0,delay_ms:20,kill_worker_after:100"
  drop_stream:p        the worker aborts a token stream with probability p per request
  fail_prefill:p       a prefill worker rejects /prefill with probability p (decode falls back locally)
  delay_ms:n           adds n ms to every engine step
  kill_worker_after:n  the worker process exits after n generated tokens
"""
from __future__ import annotations

import collections
import contextlib
import ctypes
import json
import logging
import os
import random
import threading
import time
from typing import Optional

log = logging.getLogger("mxserve.trace")


class Trace:
    __slots__ = ("request_id", "t0", "spans", "attrs")

    def __init__(self, request_id: str):
        self.request_id = request_id
        self.t0 = time.perf_counter()
        self.spans: list = []
        self.attrs: dict = {}

    def mark(self, name: str) -> None:
        self.spans.append((name, round((time.perf_counter() - self.t0) * 1e3, 3)))

    def spans_named(self, name: str) -> bool:
        return any(n == name for n, _ in self.spans)

    def to_dict(self) -> dict:
        return {"request_id": self.request_id, "spans_ms": dict(self.spans), **self.attrs}


class Tracer:
    def __init__(self, capacity: int = 1024):
        self.enabled = os.environ.get("MXS_TRACE", "0") == "1"
        self.ring: collections.deque = collections.deque(maxlen=capacity)
        self._lock = threading.Lock()

    def start(self, request_id: str) -> Trace:
        tr = Trace(request_id)
        tr.attrs["t_unix"] = round(time.time(), 3)  # wall clock of the request's arrival (window filters)
        return tr

    def finish(self, tr: Trace) -> None:
        tr.mark("done")
        d = tr.to_dict()
        with self._lock:
            self.ring.append(d)
        if self.enabled:
            log.info(json.dumps(d))

    def recent(self, n: int = 100) -> list:
        with self._lock:
            return list(self.ring)[-n:]


TRACER = Tracer()


# ----------------------------------------------------------------------------- roctx
class _Roctx:
    def __init__(self):
        self.lib = None
        if os.environ.get("MXS_ROCTX", "0") == "1":
            for name in ("libroctx64.so", "/opt/rocm/lib/libroctx64.so"):
                try:
                    self.lib = ctypes.CDLL(name)
                    break
                except OSError:
                    continue

    @contextlib.contextmanager
    def range(self, name: str):
        if self.lib is None:
            yield
            return
        self.lib.roctxRangePushA(name.encode())
        try:
            yield
        finally:
            self.lib.roctxRangePop()


ROCTX = _Roctx()


# ----------------------------------------------------------------------------- torch.profiler
class StepProfiler:
    """Python + GPU-launch view of a window of engine steps (SURVEY.md §5.1 "torch.profiler for the
    Python side"): MXS_TORCH_PROFILE="start:count:path" records steps [start, start + count) with
    torch.profiler (CPU + HIP activities) and writes a Chrome trace to `path`."""

    def __init__(self, spec: Optional[str] = None):
        spec = os.environ.get("MXS_TORCH_PROFILE", "") if spec is None else spec
        self.start = self.count = -1
        self.path = ""
        self._prof = None
        self.done = False
        if spec:
            a, b, path = spec.split(":", 2)
            self.start, self.count, self.path = int(a), int(b), path

    @property
    def enabled(self) -> bool:
        return self.count > 0 and not self.done

    def step_begin(self, step: int) -> None:
        if self.enabled and self._prof is None and step >= self.start:
            import torch
            acts = [torch.profiler.ProfilerActivity.CPU]
            if torch.cuda.is_available():
                acts.append(torch.profiler.ProfilerActivity.CUDA)
            self._prof = torch.profiler.profile(activities=acts, record_shapes=False)
            self._prof.__enter__()
            self._first = step

    def step_end(self, step: int) -> None:
        if self._prof is not None and step >= self._first + self.count - 1:
            self._prof.__exit__(None, None, None)
            self._prof.export_chrome_trace(self.path)
            log.info("torch.profiler: steps %d..%d -> %s", self._first, step, self.path)
            self._prof = None
            self.done = True


# ----------------------------------------------------------------------------- faults
class Faults:
    def __init__(self, spec: Optional[str] = None):
        spec = os.environ.get("MXS_FAULT", "") if spec is None else spec
        self.p: dict = {}
        self.args: dict = {}  # structured faults, e.g. "car_delay:rank=2:step=6:ms=1500" -> {rank: "2", ...}
        for item in filter(None, (x.strip() for x in spec.split(","))):
            k, _, v = item.partition(":")
            if "=" in v:
                self.args[k] = dict(kv.split("=", 1) for kv in v.split(":") if "=" in kv)
                continue
            self.p[k] = float(v or 1)
        self._rng = random.Random(int(os.environ.get("MXS_FAULT_SEED", "0")))
        self.tokens = 0

    def active(self) -> bool:
        return bool(self.p or self.args)

    def hit(self, name: str) -> bool:
        p = self.p.get(name, 0.0)
        return p > 0 and self._rng.random() < p

    def step_delay(self) -> None:
        d = self.p.get("delay_ms", 0.0)
        if d:
            time.sleep(d / 1e3)

    def count_tokens(self, n: int) -> None:
        lim = self.p.get("kill_worker_after")
        if lim is None:
            return
        self.tokens += n
        if self.tokens >= lim:
            log.error("fault injection: killing worker after %d tokens", self.tokens)
            os._exit(17)


FAULTS = Faults()
