"""Worker discovery + request routing (replaces etcd discovery and the Dynamo router, SURVEY.md
§2.2 X03/X06, §5.8).

Workers POST /register to the frontend and heartbeat with load + KV events; a worker that misses
its lease (ttl) is dropped.  Routing modes:
  round_robin | random | kv  -- kv = KV-aware: for each candidate worker the router knows, from the
  workers' block-stored/removed events, how many leading 16-token blocks of the prompt that worker
  already caches (native KvIndexer, csrc/runtime/block_pool.cpp).  Cost per worker:
      cost = overlap_weight * (prompt blocks still to prefill) + (active KV blocks after admission)
  normalised by the worker's pool size; lowest cost wins (ties -> fewest running requests).
  Active blocks are the worker's last report (held + its waiting queue's demand) plus the blocks of
  the requests routed to it since that report: a burst of arrivals between two heartbeats spreads
  over the workers instead of landing on the one that looked emptiest.  Workers report how many
  requests they have queued in total (num_added), which retires routed requests from that count.
  A routed request that never reaches the worker's queue (failed dispatch, rejected prompt, abort
  before admission) is retired by `forget(worker, request_id)` or, failing that, after `unseen_ttl`
  seconds; a worker whose num_added goes backwards restarted, and its unseen entries are dropped.
"""
from __future__ import annotations

import itertools
import random
import threading
import time
from collections import deque
from dataclasses import dataclass, field
from typing import Optional

from .. import _native


@dataclass
class WorkerInfo:
    worker_id: str
    url: str
    model: str
    role: str = "agg"  # agg | prefill | decode
    block_size: int = 16
    kv_total_blocks: int = 1
    tp: int = 1
    max_model_len: int = 0  # 0 = unknown
    pair: str = ""  # P/D pair pod id: a decode worker takes prefill workers of its own pair first
    stream_url: str = ""  # the worker's streamer process (token request plane), when it has one
    index: int = -1
    last_seen: float = field(default_factory=time.monotonic)
    num_running: int = 0
    num_waiting: int = 0
    kv_active_blocks: int = 0
    inflight: int = 0  # requests routed by this frontend and not finished
    kv_waiting_blocks: int = 0  # demand of the worker's waiting queue (its last report)
    num_added: int = -1  # requests the worker had queued at its last report (-1: not reported)
    # routed requests its report does not hold yet: [expiry (monotonic), blocks, request id]
    unseen: deque = field(default_factory=deque)

    def load_blocks(self, now: Optional[float] = None) -> int:
        now = time.monotonic() if now is None else now
        while self.unseen and self.unseen[0][0] <= now:  # entries are appended in expiry order
            self.unseen.popleft()
        return self.kv_active_blocks + self.kv_waiting_blocks + sum(e[1] for e in self.unseen)

    def public(self) -> dict:
        return {"worker_id": self.worker_id, "url": self.url, "model": self.model, "role": self.role,
                "kv_total_blocks": self.kv_total_blocks, "tp": self.tp, "num_running": self.num_running,
                "num_waiting": self.num_waiting, "kv_active_blocks": self.kv_active_blocks,
                "inflight": self.inflight}


class Registry:
    def __init__(self, ttl: float = 10.0, unseen_ttl: Optional[float] = None):
        self.ttl = ttl
        self.unseen_ttl = ttl if unseen_ttl is None else unseen_ttl
        self._lock = threading.Lock()
        self.workers: dict[str, WorkerInfo] = {}
        self._free_idx = list(range(63, -1, -1))
        self.indexer = _native.rt().KvIndexer()

    def register(self, info: WorkerInfo) -> WorkerInfo:
        with self._lock:
            old = self.workers.get(info.worker_id)
            if old is not None:
                info.index = old.index
            else:
                if not self._free_idx:
                    raise RuntimeError("too many workers (max 64 per frontend)")
                info.index = self._free_idx.pop()
                self.indexer.remove_worker(info.index)
            info.last_seen = time.monotonic()
            self.workers[info.worker_id] = info
            return info

    def heartbeat(self, worker_id: str, load: dict, stored=(), removed=()) -> bool:
        with self._lock:
            w = self.workers.get(worker_id)
            if w is None:
                return False
            w.last_seen = time.monotonic()
            w.num_running = int(load.get("num_running", w.num_running))
            w.num_waiting = int(load.get("num_waiting", w.num_waiting))
            tot = int(load.get("kv_total_blocks", w.kv_total_blocks) or 1)
            w.kv_total_blocks = tot
            w.kv_active_blocks = tot - int(load.get("kv_free_blocks", tot))
            w.kv_waiting_blocks = int(load.get("kv_waiting_blocks", 0))
            if "num_added" in load:
                n = int(load["num_added"])
                if 0 <= n < w.num_added:  # the worker restarted: nothing routed before is queued there
                    w.unseen.clear()
                else:
                    for _ in range(min(len(w.unseen), max(0, n - w.num_added) if w.num_added >= 0 else len(w.unseen))):
                        w.unseen.popleft()
                w.num_added = n
            else:  # a worker without the counter: its report is all the router knows
                w.unseen.clear()
            if stored:
                self.indexer.apply_stored(w.index, list(stored))
            if removed:
                self.indexer.apply_removed(w.index, list(removed))
            return True

    def deregister(self, worker_id: str) -> None:
        with self._lock:
            w = self.workers.pop(worker_id, None)
            if w is not None:
                self.indexer.remove_worker(w.index)
                self._free_idx.append(w.index)

    def expire(self) -> list[str]:
        now = time.monotonic()
        dead = [wid for wid, w in self.workers.items() if now - w.last_seen > self.ttl]
        for wid in dead:
            self.deregister(wid)
        return dead

    def list(self, model: Optional[str] = None, role: Optional[str] = None) -> list[WorkerInfo]:
        with self._lock:
            return [w for w in self.workers.values()
                    if (model is None or w.model == model) and (role is None or w.role == role)]

    def models(self) -> list[str]:
        with self._lock:
            return sorted({w.model for w in self.workers.values()})


class Router:
    def __init__(self, registry: Registry, mode: str = "kv", overlap_weight: float = 1.0, seed: int = 0):
        if mode not in ("round_robin", "random", "kv"):
            raise ValueError(f"unknown router mode {mode}")
        self.reg = registry
        self.mode = mode
        self.overlap_weight = overlap_weight
        self._rr = itertools.count()
        self._rng = random.Random(seed)
        self._hash = _native.rt().block_hashes

    def block_hashes(self, token_ids: list, block_size: int = 16) -> list:
        return self._hash(token_ids, block_size, 0, 0)

    def pick(self, candidates: list[WorkerInfo], token_ids: Optional[list] = None,
             commit: bool = True, request_id: Optional[str] = None) -> tuple[WorkerInfo, int]:
        """Returns (worker, overlap_blocks).  commit: count the request's blocks against the chosen
        worker until its load report includes them (or forget(), or the registry's unseen_ttl)."""
        w, ov = self._pick(candidates, token_ids)
        if commit and token_ids:
            bs = w.block_size
            with self.reg._lock:
                w.unseen.append([time.monotonic() + self.reg.unseen_ttl,
                                 max(0, -(-(len(token_ids) + 1) // bs) - ov), request_id])
        return w, ov

    def forget(self, w: WorkerInfo, request_id: Optional[str]) -> bool:
        """A routed request that will not be queued on w (its dispatch failed): stop counting its
        blocks against w.  The entry goes away entirely: the worker's num_added never counts it, so
        the next increments retire the requests routed after it."""
        if request_id is None:
            return False
        with self.reg._lock:
            for e in w.unseen:
                if e[2] == request_id:
                    w.unseen.remove(e)
                    return True
        return False

    def _pick(self, candidates: list[WorkerInfo], token_ids: Optional[list] = None) -> tuple[WorkerInfo, int]:
        if not candidates:
            raise LookupError("no workers available")
        if self.mode == "round_robin" or len(candidates) == 1:
            w = candidates[next(self._rr) % len(candidates)]
            return w, self._overlap(w, token_ids) if self.mode == "kv" else 0
        if self.mode == "random":
            return self._rng.choice(candidates), 0
        bs = candidates[0].block_size
        hashes = self.block_hashes(token_ids or [], bs)
        n_workers = max(w.index for w in candidates) + 1
        overlaps = self.reg.indexer.find_matches(hashes, n_workers) if hashes else [0] * n_workers
        nblocks = -(-len(token_ids or []) // bs)
        best, best_key = None, None
        for w in candidates:
            ov = overlaps[w.index]
            prefill_blocks = max(0, nblocks - ov)
            active = w.load_blocks() + nblocks
            cost = (self.overlap_weight * prefill_blocks + active) / max(1, w.kv_total_blocks)
            key = (cost, w.num_running + w.num_waiting + w.inflight, self._rng.random())
            if best_key is None or key < best_key:
                best, best_key = (w, ov), key
        return best

    def _overlap(self, w: WorkerInfo, token_ids) -> int:
        if not token_ids:
            return 0
        hashes = self.block_hashes(token_ids, w.block_size)
        return self.reg.indexer.find_matches(hashes, w.index + 1)[w.index] if hashes else 0
