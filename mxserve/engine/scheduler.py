"""Continuous-batching scheduler with chunked prefill and prefix caching (replaces the schedulers
inside the vLLM / SGLang / TRT-LLM engines the reference wraps, SURVEY.md §3.3 "ENGINE STEP LOOP").

Each step packs one token per running decode request plus prefill chunks under a token budget
(`max_num_batched_tokens`); a long prompt is split over steps so decode latency stays bounded.
When the block pool runs dry the lowest-priority (latest) running request is preempted and
recomputed later.  Decodes are ordered before prefills in the batch, which lets the model runner
use the decode attention kernel on the head of the batch and the prefill kernel on the tail.
"""
from __future__ import annotations

import time
from collections import deque
from dataclasses import dataclass, field
from typing import Optional

from .kv_manager import KVCacheManager
from .request import Request, Status


@dataclass
class ScheduledReq:
    req: Request
    num_new_tokens: int
    # sample a token at the end of this chunk (chunk reaches the end of the known tokens)
    sample: bool
    start: int = 0  # first position computed by this chunk
    out_idx: int = 0  # index of the output token this chunk samples (RNG counter)


@dataclass
class SchedulerOutput:
    decodes: list = field(default_factory=list)  # ScheduledReq, 1 token each
    prefills: list = field(default_factory=list)  # ScheduledReq, chunk of >=1 token
    preempted: list = field(default_factory=list)

    @property
    def num_tokens(self) -> int:
        return len(self.decodes) + sum(s.num_new_tokens for s in self.prefills)

    @property
    def is_empty(self) -> bool:
        return not self.decodes and not self.prefills

    def all(self):
        return self.decodes + self.prefills


class Scheduler:
    def __init__(self, kv: KVCacheManager, max_num_seqs: int = 256, max_num_batched_tokens: int = 8192,
                 max_model_len: int = 8192, enable_chunked_prefill: bool = True):
        self.kv = kv
        self.max_num_seqs = max_num_seqs
        self.max_num_batched_tokens = max_num_batched_tokens
        self.max_model_len = max_model_len
        self.chunked = enable_chunked_prefill
        self.waiting: deque[Request] = deque()
        self.running: list[Request] = []
        self.finished_ids: list[str] = []
        self.num_preemptions = 0
        # requests ever queued here (add / reserve_remote): routers match it against what they sent
        # to tell which of their routed requests this worker's load already reflects
        self.num_added = 0
        # disaggregated decode: requests whose prompt KV is being written by a prefill worker
        self.remote: dict[str, Request] = {}
        # decode-aware prefill budget (engine/pacing.py ChunkBudget), set by the engine when an
        # inter-token latency target is configured
        self.chunk_budget = None

    # ------------------------------------------------------------------ queue ops
    def add(self, req: Request) -> None:
        if req.num_prompt_tokens >= self.max_model_len:
            raise ValueError(f"prompt of {req.num_prompt_tokens} tokens exceeds max_model_len "
                             f"{self.max_model_len}")
        req.status = Status.WAITING
        self.waiting.append(req)
        self.num_added += 1

    def abort(self, request_id: str) -> Optional[Request]:
        if request_id in self.remote:
            return self.cancel_remote(request_id)
        for q in (self.running, self.waiting):
            for r in list(q):
                if r.request_id == request_id:
                    q.remove(r)
                    self._finish(r, Status.FINISHED_ABORTED)
                    return r
        return None

    def has_work(self) -> bool:
        return bool(self.waiting or self.running)

    # ------------------------------------------------------------------ disaggregation (decode side)
    def num_slots_used(self) -> int:
        """Batch rows held: running requests plus remote-prefill reservations (each becomes a
        running request when its KV lands, so both count against max_num_seqs)."""
        return len(self.running) + len(self.remote)

    def reserve_remote(self, req: Request) -> bool:
        """Allocate KV blocks for the whole prompt of a request whose prefill runs remotely.
        Locally cached prefix blocks are reused (only the rest must be transferred).  Refused
        (False) when the batch is full: the model runner has max_num_seqs rows."""
        if self.num_slots_used() >= self.max_num_seqs:
            return False
        req.num_cached_tokens = self.kv.get_computed_blocks(req)
        req.num_computed_tokens = req.num_cached_tokens
        if not self.kv.allocate_slots(req, req.num_prompt_tokens - req.num_computed_tokens):
            self.kv.free(req)
            req.num_computed_tokens = req.num_cached_tokens = 0
            return False
        req.status = Status.WAITING
        self.remote[req.request_id] = req
        self.num_added += 1
        return True

    def complete_remote(self, request_id: str, first_token: int) -> Request:
        """KV for the prompt has landed: the request joins the running batch with its first token."""
        req = self.remote.pop(request_id)
        req.num_computed_tokens = req.num_prompt_tokens
        self.kv.cache_computed_blocks(req)
        req.output_token_ids.append(int(first_token))
        req.first_token_time = time.monotonic()
        st = req.check_stop(self.max_model_len)
        if st is not None:
            self._finish(req, st)
        else:
            req.status = Status.RUNNING
            self.running.append(req)
        return req

    def cancel_remote(self, request_id: str) -> Optional[Request]:
        req = self.remote.pop(request_id, None)
        if req is not None:
            self._finish(req, Status.FINISHED_ABORTED)
        return req

    def _finish(self, req: Request, status: Status) -> None:
        req.status = status
        req.finish_time = time.monotonic()
        self.kv.free(req)

    def _preempt(self, req: Request) -> None:
        self.kv.free(req)
        req.num_computed_tokens = 0
        req.num_cached_tokens = 0
        req.status = Status.PREEMPTED
        req.num_preemptions += 1
        self.num_preemptions += 1
        self.waiting.appendleft(req)

    # ------------------------------------------------------------------ schedule
    def schedule(self) -> SchedulerOutput:
        out = SchedulerOutput()
        budget = self.max_num_batched_tokens
        scheduled: list[ScheduledReq] = []
        cb = self.chunk_budget
        left = cb.begin(self.running, self.waiting) if cb is not None else None  # seconds for prefill chunks
        first = True
        i = 0
        while i < len(self.running) and budget > 0:
            req = self.running[i]
            n = req.num_tokens - req.num_computed_tokens
            if n <= 0 or (req.num_pending and not req.can_grow(self.max_model_len)):
                i += 1
                continue
            n = min(n, budget)
            if left is not None and (n > 1 or req.num_computed_tokens < req.num_prompt_tokens):
                n, cost = cb.fit(left, req.num_computed_tokens, n, first)
                first = False
                if n <= 0:
                    i += 1
                    continue
                left -= cost
            if n < req.num_tokens - req.num_computed_tokens and not self.chunked:
                break
            while not self.kv.allocate_slots(req, n):
                victim = self.running.pop()
                if victim is req:
                    self._preempt(req)
                    out.preempted.append(req)
                    req = None
                    break
                self._preempt(victim)
                out.preempted.append(victim)
                scheduled = [s for s in scheduled if s.req is not victim]
            if req is None:
                break
            scheduled.append(ScheduledReq(req, n, req.num_computed_tokens + n >= req.num_tokens))
            budget -= n
            i += 1

        while self.waiting and budget > 0 and self.num_slots_used() < self.max_num_seqs and not out.preempted:
            req = self.waiting[0]
            if req.num_pending:  # preempted with a sample still in flight: wait for it
                break
            if req.num_computed_tokens == 0 and not req.block_ids:
                req.num_cached_tokens = self.kv.get_computed_blocks(req)
                req.num_computed_tokens = req.num_cached_tokens
            n = req.num_tokens - req.num_computed_tokens
            if n > budget:
                if not self.chunked:
                    break
                n = budget
            if left is not None and self.chunked:
                n, cost = cb.fit(left, req.num_computed_tokens, n, first)
                if n <= 0:
                    break
            if not self.kv.allocate_slots(req, n):
                # a waiting request holds no blocks: give back the cached prefix get_computed_blocks
                # pinned for it.  Kept, it stays pinned while the request waits; under overload (every
                # running request preempted, each re-queued one pinning its own cached prompt at the
                # head in turn) those pins exhausted the pool with nothing running to free it -- a
                # deadlock seen with 8 engines on one GPU (profiles/r6/overload_deadlock/)
                if req.block_ids:
                    self.kv.free(req)
                req.num_computed_tokens = req.num_cached_tokens = 0
                break
            self.waiting.popleft()
            if req.scheduled_time is None:
                req.scheduled_time = time.monotonic()
            req.status = Status.RUNNING
            self.running.append(req)
            scheduled.append(ScheduledReq(req, n, req.num_computed_tokens + n >= req.num_tokens))
            budget -= n
            if left is not None and self.chunked:
                left -= cost
                first = False

        for s in scheduled:
            r = s.req
            is_decode = s.num_new_tokens == 1 and r.num_computed_tokens >= r.num_prompt_tokens
            (out.decodes if is_decode else out.prefills).append(s)
            # advance now (not at update) so the next step can be scheduled while this one runs
            s.start = r.num_computed_tokens
            r.num_computed_tokens += s.num_new_tokens
            if s.sample:
                s.out_idx = len(r.output_token_ids) + r.num_pending
                r.num_pending += 1
        return out

    # ------------------------------------------------------------------ update
    def update(self, out: SchedulerOutput, sampled: dict[str, int]) -> list[Request]:
        """Land a step's results: register newly full blocks, append sampled tokens, retire
        finished requests.  Returns requests that produced a new token this step (finished ones
        included).  With async scheduling the next step may already be in flight; a request that
        finishes here simply has its in-flight result discarded at the next update."""
        emitted = []
        now = time.monotonic()
        bs = self.kv.block_size
        for s in out.all():
            req = s.req
            if req.is_finished:  # aborted / finished while this step was in flight
                continue
            landed = s.start + s.num_new_tokens  # KV written by THIS step (not the one in flight)
            if not s.sample:
                if min(landed, req.num_known_tokens) // bs > req.num_registered_blocks:
                    self.kv.cache_computed_blocks(req, landed)
                continue
            req.num_pending -= 1
            tok = sampled.get(req.request_id)
            if tok is None:
                continue
            req.output_token_ids.append(int(tok))
            if req.first_token_time is None:
                req.first_token_time = now
            if min(landed, req.num_known_tokens) // bs > req.num_registered_blocks:
                self.kv.cache_computed_blocks(req, landed)
            st = req.check_stop(self.max_model_len)
            if req.disagg_role == "prefill_only" and st is None:
                st = Status.FINISHED_LENGTH
            if st is not None:
                preempted = req.status == Status.PREEMPTED
                if req.disagg_role == "prefill_only":
                    # keep the blocks: the KV transfer reads them; released by release_blocks()
                    req.status = st
                    req.finish_time = now
                else:
                    self._finish(req, st)
                if preempted:
                    self.waiting.remove(req)
                else:
                    self.running.remove(req)
                self.finished_ids.append(req.request_id)
            emitted.append(req)
        return emitted

    def rewind(self, outs: list) -> int:
        """Undo launched-but-never-landed steps (their results were discarded: a collective fault).
        Each request goes back to the first position those steps computed and forgets their pending
        samples; its blocks stay allocated (the recomputation writes the same slots) and no block
        those steps wrote was registered in the prefix cache (registration happens at update).
        Returns the number of requests rewound."""
        seen = set()
        for out in outs:
            for s in out.all():
                req = s.req
                if s.sample:
                    req.num_pending = max(0, req.num_pending - 1)
                if req.is_finished:
                    continue
                req.num_computed_tokens = min(req.num_computed_tokens, s.start)
                seen.add(req.request_id)
        return len(seen)

    def release_blocks(self, req: Request) -> None:
        self.kv.free(req)

    def waiting_blocks(self) -> int:
        """KV blocks the waiting queue will take on admission (prompt + first token, uncached)."""
        bs = self.kv.block_size
        return sum(-(-(r.num_prompt_tokens + 1) // bs) for r in self.waiting)

    def stats(self) -> dict:
        return {"num_running": len(self.running), "num_waiting": len(self.waiting),
                "kv_usage": self.kv.usage(), "kv_free_blocks": self.kv.num_free(),
                "kv_total_blocks": self.kv.num_blocks, "prefix_hit_rate": self.kv.hit_rate(),
                "num_preemptions": self.num_preemptions, "num_added": self.num_added,
                "kv_waiting_blocks": self.waiting_blocks()}
