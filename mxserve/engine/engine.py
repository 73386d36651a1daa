"""LLMEngine: scheduler + KV manager + model runner, stepped synchronously; AsyncEngine runs the
step loop on a dedicated thread and fans tokens out to per-request asyncio queues (used by the
worker HTTP server and by the in-process benchmark)."""
from __future__ import annotations

import asyncio
import collections
import logging
import os
import threading
import time
import uuid
from dataclasses import dataclass
from typing import Optional

from ..config import EngineArgs
from .. import ops
from ..models.config import get_model_config
from .kv_manager import KVCacheManager
from .model_runner import ModelRunner
from ..parallel.custom_allreduce import CollectiveFault
from .request import Request, SamplingParams, Status
from .scheduler import Scheduler
from ..utils import gcpause
from ..utils.tracing import ROCTX, StepProfiler

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
    logprob: Optional[float] = None  # of token_id, when the request asked for logprobs
    top_logprobs: Optional[list] = None  # [(token_id, logprob)] best first
    timing: Optional[dict] = None  # on a request's first token: where its time to first token went


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
        self.num_collective_faults = 0  # TP steps discarded and recomputed after a custom all-reduce fault
        self.check_invariants = False
        # async scheduling: the launched-but-not-collected step (scheduler output, runner handle)
        self.async_scheduling = bool(args.async_scheduling)
        # late admission (engine/pacing.py): async steps on the GPU only, and only when the serving
        # layer provides an admit hook (AsyncEngine, bench.py)
        self.admit_hook = None
        self._late = None
        if (self.async_scheduling and self.runner.is_gpu and
                os.environ.get("MXS_LATE_ADMISSION", "1") == "1"):
            from .pacing import LateAdmission
            self._late = LateAdmission()
        self._inflight: Optional[tuple] = None
        # decode-aware prefill chunk budget (engine/pacing.py ChunkBudget): fed with every step's GPU
        # time (runner events; the step's wall time when synchronous on the CPU)
        if args.itl_target_ms and args.itl_target_ms > 0:
            from .pacing import ChunkBudget
            self.scheduler.chunk_budget = ChunkBudget(args.itl_target_ms)
        self.profiler = StepProfiler()  # MXS_TORCH_PROFILE="start:count:path"
        # MXS_STEP_TIMING=1: host seconds per phase (schedule / launch / collect wait / land)
        self.step_times: Optional[dict] = ({"schedule": 0.0, "launch": 0.0, "collect": 0.0, "land": 0.0,
                                            "steps": 0} if os.environ.get("MXS_STEP_TIMING") == "1" else None)
        # the start-up heap (torch, graphs, weights' Python side) goes to the permanent generation: a
        # full collection over it stalled the step loop ~110 ms at a time (utils/gcpause.py)
        if self.runner.is_gpu:
            gcpause.freeze_heap()

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

    # ------------------------------------------------------------------ disaggregation
    def reserve_remote_prefill(self, prompt_token_ids: list, sampling: SamplingParams,
                               request_id: str) -> Optional[Request]:
        """Decode side: allocate the prompt's blocks; None if the pool is full."""
        req = Request(request_id, list(prompt_token_ids), sampling, eos_token_ids=self.eos,
                      disagg_role="remote_prefill")
        if not self.scheduler.reserve_remote(req):
            return None
        self.requests[request_id] = req
        return req

    def complete_remote_prefill(self, request_id: str, first_token: int, logprob: Optional[float] = None,
                                top_logprobs: Optional[list] = None) -> StepOutput:
        req = self.scheduler.complete_remote(request_id, first_token)
        fin = req.is_finished
        if fin:
            self.requests.pop(request_id, None)
            self.runner.release(request_id)
        self.num_generated += 1
        return StepOutput(req.request_id, int(first_token), fin, req.status.value if fin else None,
                          req.num_prompt_tokens, req.num_cached_tokens, len(req.output_token_ids), logprob,
                          top_logprobs)

    def detach_remote_prefill(self, request_id: str) -> Optional[Request]:
        """Decode side, a remote prefill given up while its KV push may still be in flight (the
        client went away mid-transfer): forget the request -- its id is free again, e.g. for the
        local-prefill fallback -- but keep its KV blocks allocated until release_detached(), so a
        late push cannot land in blocks another request already owns."""
        req = self.scheduler.remote.pop(request_id, None)
        if req is None:
            return None
        self.requests.pop(request_id, None)
        self.runner.release(request_id)
        return req

    def release_detached(self, req: Request) -> None:
        """The prefill side is known to be done with a detached request's blocks: free them."""
        self.scheduler.release_blocks(req)

    def release_prefill_blocks(self, request_id: str) -> None:
        """Prefill side: drop the blocks kept alive for the KV transfer."""
        req = self.requests.pop(request_id, None)
        if req is not None:
            self.scheduler.release_blocks(req)

    def has_unfinished(self) -> bool:
        return self.scheduler.has_work() or self._inflight is not None

    # ------------------------------------------------------------------ step
    def step(self) -> list[StepOutput]:
        """One engine iteration.  Synchronous: schedule, run, land.  Async: schedule and launch
        step N+1 first, then land step N (whose GPU work finished while the host was busy), so the
        GPU queue never drains between steps."""
        if self.profiler.enabled:
            step_no = self.num_steps
            self.profiler.step_begin(step_no)
            try:
                return self._step()
            finally:
                self.profiler.step_end(step_no)
        return self._step()

    def _step(self) -> list[StepOutput]:
        tm = self.step_times
        late = self._late
        if late is not None and self._inflight is not None and self.admit_hook is not None:
            late.wait(self._inflight[1].get("ev"))  # until the in-flight step is nearly done
            self.admit_hook()  # requests that arrived meanwhile join the step launched next
        t_adm = time.perf_counter()
        t0 = time.perf_counter() if tm is not None else 0.0
        so = self.scheduler.schedule()
        if tm is not None:
            t1 = time.perf_counter()
            tm["schedule"] += t1 - t0
        handle = None
        t_begin = time.perf_counter()
        if not so.is_empty:
            if ROCTX.lib is not None:  # MXS_ROCTX=1: named ranges on the rocprofv3 timeline
                with ROCTX.range(f"step {self.num_steps} d{len(so.decodes)} p{len(so.prefills)}"):
                    handle = self.runner.launch(so)
            else:
                handle = self.runner.launch(so)
            kv_ev = None
            for s in so.prefills:
                self.num_prompt_computed += s.num_new_tokens
                if s.sample and s.req.disagg_role == "prefill_only" and self.runner.is_gpu:
                    if kv_ev is None:  # this step completes a prompt whose KV will be pushed
                        import torch
                        kv_ev = torch.cuda.Event()
                        kv_ev.record()
                    s.req.kv_ready = kv_ev
            self.num_steps += 1
        if tm is not None:
            t2 = time.perf_counter()
            tm["launch"] += t2 - t1
        done_state = None
        if late is not None:
            if handle is not None:
                late.launched(so, t_adm, time.perf_counter(), t_begin)
            done_state = late.inflight
            late.rotate()
        if self.async_scheduling:
            done, self._inflight = self._inflight, ((so, handle) if handle is not None else None)
        else:
            done = (so, handle) if handle is not None else None
        if done is None:
            return []
        dso, dh = done
        try:
            if late is not None:
                ev = dh.get("ev")
                pending = ev is not None and not ev.query()
                sampled = self.runner.collect(dh)
                t_done = done_state.get("done") if done_state else None
                late.observe_done(done_state, t_done if t_done is not None else
                                  (time.perf_counter() if pending else None), dh.get("gpu_s"))
            else:
                sampled = self.runner.collect(dh)
        except CollectiveFault as fault:
            return self._recover_collective_fault(dso, fault)
        cb = self.scheduler.chunk_budget
        if cb is not None:
            from .pacing import step_features
            g = dh.get("gpu_s")
            if g is None and not self.async_scheduling:
                g = time.perf_counter() - t_adm  # synchronous step: its wall time
            if g is not None:
                cb.observe(step_features(dso), g)
        if tm is None:
            return self._land(dso, sampled, dh.get("logprobs"))
        t3 = time.perf_counter()
        out = self._land(dso, sampled, dh.get("logprobs"))
        tm["collect"] += t3 - t2
        tm["land"] += time.perf_counter() - t3
        tm["steps"] += 1
        return out

    def _recover_collective_fault(self, so, fault: CollectiveFault) -> list[StepOutput]:
        """A TP collective gave up during step `so` (runner.collect raised before anything of it
        landed).  Nothing of that step, nor of the step already in flight behind it (its inputs may
        be the faulted step's tokens), reaches a client: both are drained and discarded, their
        requests rewound to the positions those steps were computing (the scheduler recomputes the
        same positions with the same sampling counters, so seeded and greedy outputs are unchanged),
        and the collective path is re-armed -- or, after repeated faults, turned off -- on every
        rank before the next step."""
        inflight, self._inflight = self._inflight, None
        steps = [so]
        if inflight is not None:
            self.runner.drain(inflight[1])
            steps.append(inflight[0])
        n = self.scheduler.rewind(steps)
        self.runner.recover_collectives(fault)
        self.num_collective_faults += 1
        if self._late is not None:
            self._late.inflight = self._late.pending_next = None
            self._late.last_done = None
        log.error("collective fault: discarded %d step(s), rewound %d request(s)", len(steps), n)
        return []

    def _land(self, so, sampled: dict, logprobs: Optional[dict] = None) -> list[StepOutput]:
        emitted = self.scheduler.update(so, sampled)
        outs = []
        for req in emitted:
            fin = req.is_finished
            lp = logprobs.get(req.request_id) if logprobs else None
            outs.append(StepOutput(req.request_id, req.output_token_ids[-1], fin,
                                   req.status.value if fin else None, req.num_prompt_tokens,
                                   req.num_cached_tokens, len(req.output_token_ids),
                                   lp[0] if lp else None, lp[1] if lp else None,
                                   _first_token_timing(req) if len(req.output_token_ids) == 1 else None))
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
        s["custom_ar_timeouts"] = self.num_collective_faults
        if self.runner.is_gpu:
            s["gemm_pf_timeouts"] = ops.gemm_pf_faults_async(self.runner.device)  # no device sync
            if s["gemm_pf_timeouts"] > getattr(self, "_pf_faults_seen", 0):
                self._pf_faults_seen = s["gemm_pf_timeouts"]
                log.error("gemm_pf: %d stream-K waits timed out (grid not resident); prefill sums of "
                          "those tiles are wrong", s["gemm_pf_timeouts"])
        la = self._late
        if la is not None:
            s["late_admission"] = {"waits": la.waits, "late_wakes": la.late, "margin_ms": round(1e3 * la.margin, 3),
                                   "host_lead_ms": round(1e3 * la.host_lead, 3), "model_updates": la.model.n}
        if self.scheduler.chunk_budget is not None:
            s["chunk_budget"] = self.scheduler.chunk_budget.stats()
        return s

    def shutdown(self) -> None:
        self.runner.shutdown_followers()

    def close(self) -> None:
        """Drop every device allocation (graphs, KV pool, weights) so another engine can be built
        in this process (bench phases)."""
        self.shutdown()
        self._inflight = None
        self.requests.clear()
        self.runner.close()
        gcpause.unfreeze_heap()  # this engine's cycles were frozen with it: collectable again


class AsyncEngine:
    """Engine loop on a dedicated thread.  The asyncio side never takes a lock that the step holds:
    commands (add / abort / disagg hooks) go through a thread-safe inbox drained by the engine
    thread between steps, and results come back through futures; tokens fan out to per-request
    asyncio queues."""

    def __init__(self, engine: LLMEngine):
        self.engine = engine
        self._inbox: collections.deque = collections.deque()
        self._wake = threading.Event()
        self._queues: dict[str, tuple[asyncio.AbstractEventLoop, asyncio.Queue]] = {}
        self._stop = False
        self.on_step = None  # optional callback(list[StepOutput]) run on the engine thread
        self._ring = None  # (cmd ring, out ring, handler): a streamer process owns the request plane
        self.last_stats: dict = engine.stats()
        self._stats_t = 0.0
        engine.admit_hook = self._admit  # late admission: arrivals up to the last moment join the next step
        self._thread = threading.Thread(target=self._loop, name="mxs-engine", daemon=True)
        self._thread.start()

    # ---------------------------------------------------------------- engine thread
    def _drain(self) -> None:
        while self._inbox:
            fn, a, kw, loop, fut = self._inbox.popleft()
            try:
                r = fn(*a, **kw)
                if fut is not None:
                    loop.call_soon_threadsafe(_set_result, fut, r, None)
            except BaseException as e:  # noqa: BLE001 - delivered to the awaiting coroutine
                if fut is not None:
                    loop.call_soon_threadsafe(_set_result, fut, None, e)
                else:
                    log.exception("engine command failed")

    def _admit(self) -> None:
        """Engine thread, right before a step is scheduled: run the commands that arrived since."""
        self._drain()
        if self._ring is not None:
            self._drain_ring(0.0)

    def _loop(self) -> None:
        while not self._stop:
            self._drain()
            if self._ring is not None:
                self._drain_ring(0.0)
            if not self.engine.has_unfinished():
                self.last_stats = self.engine.stats()
                if self._ring is not None and not self._wake.is_set():
                    self._drain_ring(0.005)  # idle: a ring command wakes the loop at once
                else:
                    self._wake.wait(0.05)
                self._wake.clear()
                continue
            try:
                outs = self.engine.step()
            except Exception:  # noqa: BLE001 - fail the in-flight requests, keep serving
                log.exception("engine step failed")
                outs = self._fail_all()
            now = time.monotonic()
            if now - self._stats_t >= 0.02:  # readers (heartbeat load, /metrics) poll far slower
                self.last_stats = self.engine.stats()
                self._stats_t = now
            if self.on_step is not None:
                try:
                    self.on_step(outs)
                except Exception:  # noqa: BLE001
                    log.exception("on_step callback failed")
            self._deliver(outs)

    def _deliver(self, outs) -> None:
        """One cross-thread wakeup per event loop per step (not per token): at ~20k tokens/s a
        call_soon_threadsafe per token costs the serving process a self-pipe write each and fights
        the engine thread for the GIL.  Requests of the streamer process (attach_ring) go out as
        ONE ring message per step, written here on the engine thread."""
        by_loop: dict = {}
        ring_outs = []
        for o in outs:
            ent = self._queues.get(o.request_id)
            if ent is None:
                continue
            loop, q = ent
            if loop is None:
                ring_outs.append(o)
            else:
                by_loop.setdefault(loop, []).append((q, o))
            if o.finished:
                self._queues.pop(o.request_id, None)
        for loop, items in by_loop.items():
            loop.call_soon_threadsafe(_put_many, items)
        if ring_outs:
            self._ring[2].emit(ring_outs)

    # ---------------------------------------------------------------- streamer process (ring)
    def attach_ring(self, handler) -> None:
        """Hand the token request plane to a streamer process (mxserve/worker/streamer.py):
        handler.poll(timeout) -> command or None, handler.command(cmd) runs it (engine thread),
        handler.emit(outs) writes one step's outputs.  Set before traffic arrives."""
        self._ring = (None, None, handler)

    def _drain_ring(self, timeout: float) -> None:
        h = self._ring[2]
        while True:
            cmd = h.poll(timeout)
            if cmd is None:
                return
            timeout = 0.0
            try:
                h.command(cmd)
            except Exception:  # noqa: BLE001 - a bad command must not stop the engine loop
                log.exception("streamer command failed")

    def own_by_ring(self, request_id: str) -> None:
        """Route this request's outputs to the streamer ring (engine thread or before the loop sees it)."""
        self._queues[request_id] = (None, None)

    def _fail_all(self) -> list:
        self.engine._inflight = None  # the failed step's results are never collected
        outs = []
        for rid in list(self.engine.requests):
            self.engine.abort(rid)
            outs.append(StepOutput(rid, -1, True, "error", 0, 0, 0))
        return outs

    # ---------------------------------------------------------------- asyncio side
    def submit(self, fn, *a, **kw) -> asyncio.Future:
        loop = asyncio.get_running_loop()
        fut = loop.create_future()
        self._inbox.append((fn, a, kw, loop, fut))
        self._wake.set()
        return fut

    def submit_nowait(self, fn, *a, **kw) -> None:
        self._inbox.append((fn, a, kw, None, None))
        self._wake.set()

    def open_stream(self, request_id: str) -> asyncio.Queue:
        q: asyncio.Queue = asyncio.Queue()
        self._queues[request_id] = (asyncio.get_running_loop(), q)
        return q

    def push(self, out: StepOutput) -> None:
        """Deliver an output produced outside a step (e.g. a remotely prefilled first token).  With a
        streamer ring the engine thread is the ring's only producer: queue it there."""
        if self._ring is not None and threading.current_thread() is not self._thread:
            self.submit_nowait(self._deliver, [out])
        else:
            self._deliver([out])

    async def stream(self, request_id: str, q: asyncio.Queue):
        try:
            while True:
                o = await q.get()
                yield o
                if o.finished:
                    return
        finally:
            if self._queues.pop(request_id, None) is not None:  # client went away mid-stream
                self.submit_nowait(self.engine.abort, request_id)

    async def stream_batches(self, request_id: str, q: asyncio.Queue):
        """Like stream(), but yields every output already queued at once (a list)."""
        try:
            while True:
                outs = [await q.get()]
                while not outs[-1].finished and not q.empty():
                    outs.append(q.get_nowait())
                yield outs
                if outs[-1].finished:
                    return
        finally:
            if self._queues.pop(request_id, None) is not None:  # client went away mid-stream
                self.submit_nowait(self.engine.abort, request_id)

    async def generate(self, prompt_token_ids: list, sampling: SamplingParams, request_id: Optional[str] = None,
                       disagg_role: Optional[str] = None):
        """Async iterator of StepOutput for one request."""
        rid = request_id or uuid.uuid4().hex
        q = self.open_stream(rid)
        try:
            await self.submit(self.engine.add_request, prompt_token_ids, sampling, rid, disagg_role)
        except BaseException:
            self._queues.pop(rid, None)
            raise
        async for o in self.stream(rid, q):
            yield o

    def shutdown(self) -> None:
        self._stop = True
        self._wake.set()
        self._thread.join(timeout=5)


def _first_token_timing(req) -> dict:
    """Worker-side spans of a request's time to first token (ms): waiting for admission, then the
    prefill steps up to the sampled token."""
    sched = req.scheduled_time if req.scheduled_time is not None else req.arrival_time
    first = req.first_token_time if req.first_token_time is not None else sched
    t = {"queue_ms": round((sched - req.arrival_time) * 1e3, 3), "prefill_ms": round((first - sched) * 1e3, 3),
         "emit_unix": time.time()}  # the consumer's receive time minus this = delivery latency (same host)
    if req.submit_time is not None:  # waiting in the engine thread's inbox for a step boundary
        t["inbox_ms"] = round((req.arrival_time - req.submit_time) * 1e3, 3)
    return t


def _put_many(items: list) -> None:
    for q, o in items:
        q.put_nowait(o)


def _set_result(fut: asyncio.Future, r, e) -> None:
    if fut.done():
        return
    if e is not None:
        fut.set_exception(e)
    else:
        fut.set_result(r)


def now() -> float:
    return time.monotonic()


__all__ = ["LLMEngine", "AsyncEngine", "StepOutput", "SamplingParams", "Status"]
