"""LLMEngine: scheduler + KV manager + model runner, stepped synchronously; AsyncEngine runs the
step loop on a dedicated thread and fans tokens out to per-request asyncio queues (used by the
worker HTTP server and by the in-process benchmark)."""
from __future__ import annotations

import asyncio
import logging
import threading
import time
import uuid
from dataclasses import dataclass
from typing import Optional

from ..config import EngineArgs
from ..models.config import get_model_config
from .kv_manager import KVCacheManager
from .model_runner import ModelRunner
from .request import Request, SamplingParams, Status
from .scheduler import Scheduler

log = logging.getLogger(__name__)


@dataclass
class StepOutput:
    request_id: str
    token_id: int
    finished: bool
    finish_reason: Optional[str]
    num_prompt_tokens: int
    num_cached_tokens: int
    num_output_tokens: int


class LLMEngine:
    def __init__(self, args: EngineArgs):
        self.args = args
        self.model_config = get_model_config(args.model)
        self.runner = ModelRunner(args, self.model_config)
        self.kv = KVCacheManager(self.runner.num_blocks, args.block_size, args.enable_prefix_caching)
        self.scheduler = Scheduler(self.kv, args.max_num_seqs, args.max_num_batched_tokens, args.max_model_len,
                                   args.enable_chunked_prefill)
        self.requests: dict[str, Request] = {}
        self.eos = tuple(self.model_config.eos_token_ids)
        self.num_steps = 0
        self.num_generated = 0
        self.num_prompt_computed = 0
        self.check_invariants = False

    # ------------------------------------------------------------------ requests
    def add_request(self, prompt_token_ids: list, sampling: Optional[SamplingParams] = None,
                    request_id: Optional[str] = None, disagg_role: Optional[str] = None) -> Request:
        rid = request_id or uuid.uuid4().hex
        if rid in self.requests:
            raise ValueError(f"duplicate request id {rid}")
        req = Request(rid, list(prompt_token_ids), sampling or SamplingParams(), eos_token_ids=self.eos,
                      disagg_role=disagg_role)
        self.scheduler.add(req)
        self.requests[rid] = req
        return req

    def abort(self, request_id: str) -> None:
        req = self.scheduler.abort(request_id)
        if req is None:
            req = self.requests.get(request_id)
            if req is not None and req.block_ids:
                self.scheduler.release_blocks(req)
        self.requests.pop(request_id, None)
        self.runner.release(request_id)

    def has_unfinished(self) -> bool:
        return self.scheduler.has_work()

    # ------------------------------------------------------------------ step
    def step(self) -> list[StepOutput]:
        so = self.scheduler.schedule()
        if so.is_empty:
            return []
        sampled = self.runner.execute(so)
        for s in so.prefills:
            self.num_prompt_computed += s.num_new_tokens
        emitted = self.scheduler.update(so, sampled)
        self.num_steps += 1
        outs = []
        for req in emitted:
            fin = req.is_finished
            outs.append(StepOutput(req.request_id, req.output_token_ids[-1], fin,
                                   req.status.value if fin else None, req.num_prompt_tokens,
                                   req.num_cached_tokens, len(req.output_token_ids)))
            self.num_generated += 1
            if fin:
                self.runner.release(req.request_id)
                if req.disagg_role != "prefill_only":
                    self.requests.pop(req.request_id, None)
        if self.check_invariants:
            assert self.kv.check_invariants(), "block pool invariants violated"
        return outs

    def generate(self, prompts: list, sampling: SamplingParams) -> list[list[int]]:
        """Offline batch generation (tests / benchmarks)."""
        reqs = [self.add_request(p, sampling) for p in prompts]
        while self.has_unfinished():
            self.step()
        return [r.output_token_ids for r in reqs]

    def stats(self) -> dict:
        s = self.scheduler.stats()
        s.update(num_steps=self.num_steps, num_generated=self.num_generated, **self.runner.kv_stats())
        return s

    def shutdown(self) -> None:
        self.runner.shutdown_followers()


class AsyncEngine:
    """Thread-driven engine loop with asyncio fan-out."""

    def __init__(self, engine: LLMEngine):
        self.engine = engine
        self._lock = threading.Lock()
        self._wake = threading.Event()
        self._queues: dict[str, tuple[asyncio.AbstractEventLoop, asyncio.Queue]] = {}
        self._stop = False
        self._thread = threading.Thread(target=self._loop, name="mxs-engine", daemon=True)
        self.on_step = None  # optional callback(list[StepOutput])
        self._thread.start()

    def _loop(self) -> None:
        while not self._stop:
            with self._lock:
                busy = self.engine.has_unfinished()
                outs = self.engine.step() if busy else []
            if not busy:
                self._wake.wait(0.05)
                self._wake.clear()
                continue
            if self.on_step is not None:
                try:
                    self.on_step(outs)
                except Exception:  # noqa: BLE001
                    log.exception("on_step callback failed")
            for o in outs:
                ent = self._queues.get(o.request_id)
                if ent is None:
                    continue
                loop, q = ent
                loop.call_soon_threadsafe(q.put_nowait, o)
                if o.finished:
                    self._queues.pop(o.request_id, None)

    async def generate(self, prompt_token_ids: list, sampling: SamplingParams, request_id: Optional[str] = None,
                       disagg_role: Optional[str] = None):
        """Async iterator of StepOutput for one request."""
        rid = request_id or uuid.uuid4().hex
        q: asyncio.Queue = asyncio.Queue()
        self._queues[rid] = (asyncio.get_running_loop(), q)
        with self._lock:
            self.engine.add_request(prompt_token_ids, sampling, rid, disagg_role)
        self._wake.set()
        try:
            while True:
                o = await q.get()
                yield o
                if o.finished:
                    return
        finally:
            if self._queues.pop(rid, None) is not None:
                with self._lock:
                    self.engine.abort(rid)

    def run_locked(self, fn, *a, **kw):
        with self._lock:
            return fn(*a, **kw)

    def shutdown(self) -> None:
        self._stop = True
        self._wake.set()
        self._thread.join(timeout=5)


def now() -> float:
    return time.monotonic()


__all__ = ["LLMEngine", "AsyncEngine", "StepOutput", "SamplingParams", "Status"]
