"""OpenAI-compatible HTTP frontend (replaces the Dynamo frontend: componentType frontend,
examples/deploy/vllm/agg.yaml:12-17; port 8000, README.md:260).

  GET  /v1/models                 {object: list, data: [{id, object: model, ...}]}
  POST /v1/chat/completions       chat template -> tokens -> router -> worker stream (SSE or unary)
  POST /v1/completions            same for raw prompts
  GET  /health /live /metrics     readiness = at least one worker registered; dynamo_frontend_* metrics
  POST /internal/register|heartbeat, GET /internal/workers   discovery (replaces etcd)

Errors are `{"error": {"message": ...}}` (multi_convos_parallel.sh:44-45); `Authorization` is
accepted and ignored (chat.sh:89).  The frontend tokenizes (workers run with
--skip-tokenizer-init semantics), streams incremental detokenized text, applies stop strings,
and retries a request on another worker if its worker fails before the first token.
"""
from __future__ import annotations

import asyncio
import contextvars
import contextlib
import json
import logging
import os
import time
import uuid
from dataclasses import dataclass
from typing import AsyncIterator, Optional

from fastapi import FastAPI, Request as HTTPRequest
from fastapi.responses import JSONResponse, Response, StreamingResponse

from ..models.config import find_local_model_dir, get_model_config
from ..router.router import Registry, Router, WorkerInfo
from ..utils.tracing import TRACER
from .chat_template import render
from .metrics import FrontendMetrics
from .reasoning import ReasoningSplitter, split_text
from .tokenizer import IncrementalDetokenizer, load_tokenizer

log = logging.getLogger("mxserve.frontend")


MAX_N = 16  # choices per request (`n`)


def _parse_token_line(d: dict, out: list) -> None:
    """One NDJSON line of the worker's /generate stream -> TokenEvents (a line holds one token, or a
    list of every token that was ready when the worker wrote it)."""
    toks = d["t"]
    if not isinstance(toks, list):
        if toks == -2:  # the worker dropped the stream (fault injection on the mux plane)
            raise ConnectionError("worker dropped the stream")
        if toks < 0:
            raise RuntimeError("worker failed the request")
        out.append(TokenEvent(toks, d["f"], d["r"], d["p"], d["c"], d.get("lp"), d.get("tlp"), d.get("tm")))
        return
    n = len(toks)
    lps, tlps = d.get("lp") or [None] * n, d.get("tlp") or [None] * n
    for i, t in enumerate(toks):
        if t == -2:
            raise ConnectionError("worker dropped the stream")
        if t < 0:
            raise RuntimeError("worker failed the request")
        last = i == n - 1
        out.append(TokenEvent(t, d["f"] and last, d["r"] if last else None, d["p"], d["c"], lps[i], tlps[i],
                              d.get("tm") if i == 0 else None))


def _observe_zeros(hist_child, k: int) -> None:
    """k observations of 0.0 in one histogram child: one bucket increment instead of k observe()
    calls (prometheus_client keeps a child's bucket counters in `_buckets`, lowest bound first)."""
    b = getattr(hist_child, "_buckets", None)
    if b:
        b[0].inc(k)
    else:  # pragma: no cover - other client versions
        for _ in range(k):
            hist_child.observe(0.0)


async def _merge(gens: list):
    """Interleave async generators as items arrive: yields (generator index, item).  The first
    exception ends the merge and is raised; the other generators are closed."""
    if len(gens) == 1:
        async for item in gens[0]:
            yield 0, item
        return
    q: asyncio.Queue = asyncio.Queue()
    done = object()

    async def pump(i, g):
        try:
            async for item in g:
                await q.put((i, item))
            await q.put((i, done))
        except BaseException as e:  # noqa: BLE001 - re-raised by the consumer
            await q.put((i, e))

    tasks = [asyncio.ensure_future(pump(i, g)) for i, g in enumerate(gens)]
    try:
        left = len(gens)
        while left:
            i, item = await q.get()
            if item is done:
                left -= 1
            elif isinstance(item, BaseException):
                raise item
            else:
                yield i, item
    finally:
        for t in tasks:
            t.cancel()


REQUEST_PLANE = os.environ.get("MXS_REQUEST_PLANE", "mux")  # mux | stream


class MuxClient:
    """This frontend process's end of one worker's multiplexed request plane (worker/server.py
    POST /mux): one long-lived NDJSON channel carries the tokens of every request this process sends
    to the worker, one line per engine step, demultiplexed here into per-request queues.  Requests
    join with POST /submit and leave early with POST /abort.  If the channel breaks, every request
    on it sees a ConnectionError (retry / migration, as for a broken /generate stream)."""

    HELLO_TIMEOUT = 10.0

    def __init__(self, url: str):
        self.url = url.rstrip("/")
        self.sid = uuid.uuid4().hex
        self.queues: dict[str, asyncio.Queue] = {}
        self.task: Optional[asyncio.Task] = None
        self.ready: Optional[asyncio.Future] = None
        self.unsupported = False  # the worker has no /mux: use /generate streams

    async def ensure(self, sess) -> None:
        if self.task is None or self.task.done():
            self.ready = asyncio.get_running_loop().create_future()
            self.queues = {}  # this channel's requests (the old channel fails only its own)
            self.task = asyncio.ensure_future(self._read(sess, self.ready, self.queues))
        await asyncio.wait_for(asyncio.shield(self.ready), self.HELLO_TIMEOUT)

    def reset(self) -> None:
        if self.task is not None and not self.task.done():
            self.task.cancel()
        self.task = None

    async def _read(self, sess, ready: asyncio.Future, queues: dict) -> None:
        err: BaseException = ConnectionError(f"request channel to {self.url} closed")
        try:
            async with sess.post(self.url + "/mux", json={"sid": self.sid}) as r:
                if r.status == 404:
                    self.unsupported = True
                if r.status != 200:
                    raise ConnectionError(f"request channel to {self.url}: HTTP {r.status}")
                buf = b""
                async for data in r.content.iter_any():
                    buf += data
                    *lines, buf = buf.split(b"\n")
                    for line in lines:
                        if not line:
                            continue
                        d = json.loads(line)
                        b = d.get("b")
                        if b is None:
                            if "hello" in d and not ready.done():
                                ready.set_result(True)
                            continue
                        for rid, payload in b:
                            q = queues.get(rid)
                            if q is not None:
                                q.put_nowait(payload)
        except asyncio.CancelledError:
            err = ConnectionError(f"request channel to {self.url} closed")
            raise
        except BaseException as e:  # noqa: BLE001 - handed to every request on the channel
            err = e if isinstance(e, _STREAM_ERRORS) else ConnectionError(f"request channel failed: {e!r}")
        finally:
            if not ready.done():
                ready.set_exception(err)
            for q in queues.values():
                q.put_nowait(err)
            queues.clear()


class _PushSink:
    """Stands in for a request's queue in MuxClient.queues: the channel reader's put_nowait(line)
    runs the request's PushStream right there (fastpath.py); the end or a failure resolves `fut`."""
    __slots__ = ("ps", "fut")

    def __init__(self, ps, fut: asyncio.Future):
        self.ps, self.fut = ps, fut

    def put_nowait(self, item) -> None:
        if self.fut.done():
            return
        if isinstance(item, BaseException):
            self.fut.set_exception(item)
            return
        try:
            if self.ps.on_payload(item):
                self.fut.set_result(True)
        except BaseException as e:  # noqa: BLE001 - the request's coroutine handles it
            self.fut.set_exception(e)


class APIError(Exception):
    def __init__(self, status: int, message: str, etype: str = "invalid_request_error"):
        super().__init__(message)
        self.status, self.message, self.etype = status, message, etype


def _err(status: int, message: str, etype: str = "invalid_request_error") -> JSONResponse:
    return JSONResponse({"error": {"message": message, "type": etype, "code": status}}, status_code=status)


try:  # a stream cut mid-body surfaces as aiohttp.ClientPayloadError, not a ConnectionError
    import aiohttp as _aiohttp
    _STREAM_ERRORS = (ConnectionError, OSError, asyncio.TimeoutError, _aiohttp.ClientError)
except ImportError:  # pragma: no cover
    _STREAM_ERRORS = (ConnectionError, OSError, asyncio.TimeoutError)


@dataclass
class TokenEvent:
    token_id: int
    finished: bool
    finish_reason: Optional[str]
    num_prompt_tokens: int
    num_cached_tokens: int
    logprob: Optional[float] = None
    top_logprobs: Optional[list] = None  # [(token_id, logprob)]
    timing: Optional[dict] = None  # worker-side spans of the time to first token (first event)


# the request trace of the task serving a request (route / first-token marks deeper in the stack)
_TRACE: contextvars.ContextVar = contextvars.ContextVar("mxs_trace", default=None)


class LocalWorker:
    """In-process worker (single-process serving: frontend + engine, no HTTP hop)."""

    def __init__(self, aeng, model: str):
        self.aeng = aeng
        self.model = model

    async def generate(self, token_ids, sampling: dict, request_id: str, prefill_url=None) -> AsyncIterator[list]:
        from ..worker.server import _sampling
        q = self.aeng.open_stream(request_id)
        try:
            await self.aeng.submit(self.aeng.engine.add_request, token_ids, _sampling(sampling), request_id, None)
        except BaseException:
            self.aeng._queues.pop(request_id, None)
            raise
        async for outs in self.aeng.stream_batches(request_id, q):
            yield [TokenEvent(o.token_id, o.finished, o.finish_reason, o.num_prompt_tokens, o.num_cached_tokens,
                              o.logprob, o.top_logprobs, o.timing) for o in outs]


class Frontend:
    def __init__(self, router_mode: str = "kv", ttl: float = 10.0, namespace: str = "default",
                 migrate: bool = True, reasoning_parser: Optional[str] = None):
        self.registry = Registry(ttl=ttl)
        # chat completions: split <think> blocks into `reasoning_content` (qwen3 | basic | deepseek_r1)
        self.reasoning_parser = reasoning_parser or os.environ.get("MXS_REASONING_PARSER") or None
        if self.reasoning_parser:
            ReasoningSplitter(self.reasoning_parser)  # validate the name at startup
        self.migrate = migrate  # move a broken stream to another worker (prompt + generated re-prefilled)
        self.router = Router(self.registry, router_mode)
        self.metrics = FrontendMetrics()
        self.namespace = namespace
        self._tok = {}
        self._cfg = {}
        self.local: dict[str, LocalWorker] = {}
        self._mux: dict[str, MuxClient] = {}
        self.bus = None  # multi-process frontend: discovery messages to/from the sibling processes
        self._bg: set = set()  # fire-and-forget tasks (aborts), referenced until done
        self._http = None
        self.started = time.time()
        self.app = self._build_app()

    # ---------------------------------------------------------------- discovery
    def apply_register(self, d: dict) -> WorkerInfo:
        info = WorkerInfo(worker_id=d["worker_id"], url=d["url"], model=d["model"], role=d.get("role", "agg"),
                          block_size=int(d.get("block_size", 16)),
                          kv_total_blocks=int(d.get("kv_total_blocks", 1) or 1), tp=int(d.get("tp", 1)),
                          max_model_len=int(d.get("max_model_len", 0) or 0), pair=str(d.get("pair") or ""),
                          stream_url=str(d.get("stream_url") or ""))
        self.registry.register(info)
        log.info("registered worker %s (%s) for %s at %s", info.worker_id, info.role, info.model, info.url)
        return info

    def apply_heartbeat(self, d: dict) -> bool:
        return self.registry.heartbeat(d["worker_id"], d.get("load", {}), d.get("stored", ()), d.get("removed", ()))

    def apply_peer(self, kind: str, d: dict) -> None:
        """A discovery message another process of this frontend received (frontend/multiproc.py)."""
        try:
            if kind == "register":
                self.apply_register(d)
            elif kind == "heartbeat":
                self.apply_heartbeat(d)
        except Exception:  # noqa: BLE001
            log.exception("bad peer discovery message")

    # ---------------------------------------------------------------- model info
    def tokenizer(self, model: str):
        if model not in self._tok:
            cfg = get_model_config(model)
            self._cfg[model] = cfg
            self._tok[model] = load_tokenizer(cfg)
        return self._tok[model]

    def model_cfg(self, model: str):
        self.tokenizer(model)
        return self._cfg[model]

    def add_local_worker(self, aeng, model: str, kv_total_blocks: int) -> None:
        self.local[model] = LocalWorker(aeng, model)
        self.registry.register(WorkerInfo(worker_id=f"local-{model}", url="local://", model=model,
                                          kv_total_blocks=kv_total_blocks,
                                          max_model_len=aeng.engine.args.max_model_len))
        self.registry.workers[f"local-{model}"].last_seen = float("inf")

    def resolve_model(self, name: Optional[str]) -> str:
        models = self.registry.models()
        if name in models:
            return name
        if name:
            base = name.rstrip("/").split("/")[-1].lower()
            for m in models:
                if m.rstrip("/").split("/")[-1].lower() == base:
                    return m
        if not name and len(models) == 1:
            return models[0]
        raise APIError(404, f"The model `{name}` does not exist." if name else "model is required",
                       "model_not_found")

    async def http(self):
        if self._http is None:
            import aiohttp
            self._http = aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=None, sock_connect=5),
                                               connector=aiohttp.TCPConnector(limit=0))
        return self._http

    # ---------------------------------------------------------------- request plane
    async def _worker_stream(self, w: WorkerInfo, token_ids, sampling: dict, rid: str,
                             prefill_url: Optional[str]) -> AsyncIterator[list]:
        """Yields LISTS of TokenEvent: everything that arrived since the last read.  While the
        frontend keeps up that is one token; when it falls behind, a batch flows through the rest of
        the pipeline (detokenize, one SSE chunk) at the cost of one."""
        if w.url.startswith("local://"):
            async for evs in self.local[w.model].generate(token_ids, sampling, rid, prefill_url):
                yield evs
            return
        sess = await self.http()
        body = {"request_id": rid, "token_ids": token_ids, "sampling": sampling}
        if prefill_url:
            body["prefill_url"] = prefill_url
        if REQUEST_PLANE == "mux":
            murl = w.stream_url or w.url  # the worker's streamer process, if it runs one
            mc = self._mux.get(murl)
            if mc is None:
                mc = self._mux[murl] = MuxClient(murl)
            if not mc.unsupported:
                try:
                    await mc.ensure(sess)
                except _STREAM_ERRORS:
                    if not mc.unsupported:
                        raise
                if not mc.unsupported:
                    async for evs in self._mux_stream(sess, mc, body, rid):
                        yield evs
                    return
        async with sess.post(w.url.rstrip("/") + "/generate", json=body) as r:
            if r.status != 200:
                raise ConnectionError(f"worker {w.worker_id} returned {r.status}")
            buf = b""
            async for data in r.content.iter_any():
                buf += data
                *lines, buf = buf.split(b"\n")
                evs, err = [], None
                try:
                    for line in lines:
                        if line.strip():
                            _parse_token_line(json.loads(line), evs)
                except (ConnectionError, RuntimeError) as e:
                    err = e  # the tokens before the marker still count as generated (migration, router)
                if evs:
                    yield evs
                if err is not None:
                    raise err
            if buf.strip():
                evs, err = [], None
                try:
                    _parse_token_line(json.loads(buf), evs)
                except (ConnectionError, RuntimeError) as e:
                    err = e
                if evs:
                    yield evs
                if err is not None:
                    raise err

    async def _mux_stream(self, sess, mc: MuxClient, body: dict, rid: str) -> AsyncIterator[list]:
        q: asyncio.Queue = asyncio.Queue()
        mc.queues[rid] = q
        done = False
        try:
            for attempt in range(2):
                async with sess.post(mc.url + "/submit", json=dict(body, sid=mc.sid)) as r:
                    status = r.status
                if status == 404 and attempt == 0:  # the worker restarted and lost this channel: reopen
                    mc.queues.pop(rid, None)
                    mc.reset()
                    await mc.ensure(sess)
                    q = asyncio.Queue()
                    mc.queues[rid] = q
                    continue
                if status != 200:
                    raise ConnectionError(f"submit to {mc.url} returned {status}")
                break
            while True:
                item = await q.get()
                if isinstance(item, BaseException):
                    raise item
                evs: list = []
                err = None
                try:
                    _parse_token_line(item, evs)
                    while not evs[-1].finished and not q.empty():
                        item = q.get_nowait()
                        if isinstance(item, BaseException):
                            raise item
                        _parse_token_line(item, evs)
                except (ConnectionError, RuntimeError) as e:
                    err = e  # deliver the tokens that came before the failure first
                if evs and evs[-1].finished:
                    done = True
                if evs:
                    yield evs
                if err is not None:
                    raise err
                if done:
                    return
        finally:
            mc.queues.pop(rid, None)
            if not done:  # client gone, or the stream failed: free the worker's slot
                t = asyncio.ensure_future(self._post_abort(sess, mc.url, rid))
                self._bg.add(t)
                t.add_done_callback(self._bg.discard)

    @staticmethod
    async def _post_abort(sess, url: str, rid: str) -> None:
        try:
            async with sess.post(url + "/abort", json={"request_id": rid}) as r:
                await r.read()
        except Exception:  # noqa: BLE001 - the worker is gone: nothing to free
            pass

    async def generate_tokens(self, model: str, token_ids: list, sampling: dict, rid: str) -> AsyncIterator[TokenEvent]:
        """Route + stream.  A worker that fails before the first token is retried elsewhere; one that
        fails MID-stream (connection lost, stream cut without a final event) is migrated: another
        worker re-prefills prompt + the tokens generated so far and continues with the remaining
        budget, so the client sees one uninterrupted stream."""
        tried: set = set()
        generated: list = []
        for attempt in range(4):
            pick = self._choose(model, token_ids, sampling, generated, tried, attempt, rid)
            if pick is None:
                break
            w, ids, sp, purl = pick
            w.inflight += 1
            n0 = len(generated)
            try:
                async for evs in self._worker_stream(w, ids, sp, rid, purl):
                    generated.extend(ev.token_id for ev in evs)
                    yield evs
                    if evs[-1].finished:
                        return
                raise ConnectionError(f"worker {w.worker_id} ended the stream early")
            except _STREAM_ERRORS as e:
                if len(generated) == n0:  # never reached the worker's queue: stop counting it there
                    self.router.forget(w, rid)
                self._attempt_failed(model, w, e, generated, tried)
            finally:
                w.inflight -= 1
        self._no_worker_left(model, generated, tried)

    # ---------------------------------------------------------------- push path (fastpath.py)
    async def run_push(self, model: str, token_ids: list, sampling: dict, rid: str, ps) -> None:
        """Route + stream one request into a fastpath.PushStream: the retry / migration policy of
        generate_tokens, with the tokens pushed to `ps.on_events` by the channel reader."""
        tried: set = set()
        generated = ps.generated
        for attempt in range(4):
            pick = self._choose(model, token_ids, sampling, generated, tried, attempt, rid)
            if pick is None:
                break
            w, ids, sp, purl = pick
            w.inflight += 1
            n0 = len(generated)
            try:
                await self._push_attempt(w, ids, sp, rid, purl, ps)
                return
            except _STREAM_ERRORS as e:
                from .fastpath import ClientGone
                if isinstance(e, ClientGone):  # nobody to stream to: no retry
                    raise
                # a failure after tokens arrived: the worker queued it, and its num_added (or the
                # unseen TTL) retires the entry -- forgetting here would retire a later request's
                if len(generated) == n0:
                    self.router.forget(w, rid)
                self._attempt_failed(model, w, e, generated, tried)
            finally:
                w.inflight -= 1
        self._no_worker_left(model, generated, tried)

    async def _push_attempt(self, w: WorkerInfo, ids: list, sp: dict, rid: str, purl: Optional[str], ps) -> None:
        sess = await self.http()
        body = {"request_id": rid, "token_ids": ids, "sampling": sp}
        if purl:
            body["prefill_url"] = purl
        murl = w.stream_url or w.url
        mc = self._mux.get(murl) if REQUEST_PLANE == "mux" and not w.url.startswith("local://") else None
        if mc is None and REQUEST_PLANE == "mux" and not w.url.startswith("local://"):
            mc = self._mux[murl] = MuxClient(murl)
        if mc is not None and not mc.unsupported:
            try:
                await mc.ensure(sess)
            except _STREAM_ERRORS:
                if not mc.unsupported:
                    raise
        if mc is None or mc.unsupported:  # a worker without the mux plane: pull its stream here
            async for evs in self._worker_stream(w, ids, sp, rid, purl):
                if ps.on_events(evs):
                    return
            raise ConnectionError(f"worker {w.worker_id} ended the stream early")
        fut = asyncio.get_running_loop().create_future()
        sink = _PushSink(ps, fut)
        mc.queues[rid] = sink
        tr = getattr(ps, "trace", None)
        try:
            if tr is not None and not tr.spans_named("dispatched"):
                tr.mark("dispatched")  # routed, channel open: the submit POST starts
            for attempt in range(2):
                async with sess.post(mc.url + "/submit", json=dict(body, sid=mc.sid)) as r:
                    status = r.status
                if status == 404 and attempt == 0:  # the worker restarted and lost this channel: reopen
                    mc.queues.pop(rid, None)
                    mc.reset()
                    await mc.ensure(sess)
                    mc.queues[rid] = sink
                    continue
                if status != 200:
                    raise ConnectionError(f"submit to {mc.url} returned {status}")
                break
            if tr is not None and not tr.spans_named("submitted"):
                tr.mark("submitted")  # the worker's streamer accepted it (its command is in the engine's ring)
            await fut
        finally:
            mc.queues.pop(rid, None)
            if not ps.worker_done:  # stop string, client gone or failure: free the worker's slot
                t = asyncio.ensure_future(self._post_abort(sess, mc.url, rid))
                self._bg.add(t)
                t.add_done_callback(self._bg.discard)

    def _choose(self, model: str, token_ids: list, sampling: dict, generated: list, tried: set, attempt: int,
                rid: Optional[str] = None):
        """(decode / agg worker, token ids, sampling, prefill URL) of the next attempt, or None: the
        router's pick among the workers not tried yet; after a failure mid-stream the ids are prompt +
        generated and the budget what is left (migration).  A decode worker gets a prefill worker of
        its own P/D group pod first (that one can reach its GPU arena)."""
        decode = [w for w in self.registry.list(model) if w.role in ("agg", "decode") and w.worker_id not in tried]
        prefill = [w for w in self.registry.list(model, "prefill")]
        if not decode:
            return None
        ids = token_ids + generated
        sp = sampling
        if generated:
            sp = dict(sampling, max_tokens=int(sampling.get("max_tokens", 16)) - len(generated),
                      min_tokens=max(0, int(sampling.get("min_tokens") or 0) - len(generated)))
        w, overlap = self.router.pick(decode, ids, request_id=rid)
        tr = _TRACE.get()
        if tr is not None and attempt == 0:
            tr.mark("routed")
            tr.attrs["worker"] = w.worker_id
        purl = None
        if w.role == "decode" and prefill:
            mates = [p for p in prefill if w.pair and p.pair == w.pair]
            pw, _ = self.router.pick(mates or prefill, ids)
            purl = pw.url
        if overlap:
            self.metrics.kv_hit.labels(model).inc(overlap)
        return w, ids, sp, purl

    def _attempt_failed(self, model: str, w: WorkerInfo, e: BaseException, generated: list, tried: set) -> None:
        if generated and not self.migrate:
            raise e
        log.warning("worker %s failed after %d tokens (%r); %s", w.worker_id, len(generated), e,
                    "migrating" if generated else "retrying")
        if generated:
            self.metrics.migrations.labels(model).inc()
        tried.add(w.worker_id)
        try:
            import aiohttp
            if isinstance(e, aiohttp.ClientConnectionError) and not generated:
                self.registry.deregister(w.worker_id)
        except ImportError:
            pass

    @staticmethod
    def _no_worker_left(model: str, generated: list, tried: set) -> None:
        if generated:
            raise ConnectionError("request could not be migrated: no other worker")
        raise APIError(503, f"no workers available for model {model}" if not tried else "all workers failed",
                       "service_unavailable")

    # ---------------------------------------------------------------- OpenAI layer
    def context_limit(self, model: str) -> int:
        lens = [w.max_model_len for w in self.registry.list(model) if w.max_model_len > 0]
        return min(lens) if lens else self.model_cfg(model).max_position_embeddings

    @staticmethod
    def _logprobs_arg(body: dict, chat: bool) -> Optional[int]:
        """OpenAI: chat `logprobs: bool` + `top_logprobs: 0..20`; completions `logprobs: int`."""
        if chat:
            top = body.get("top_logprobs")
            if not body.get("logprobs"):
                if top:
                    raise APIError(400, "top_logprobs requires logprobs to be true")
                return None
            k = int(top or 0)
        else:
            if body.get("logprobs") is None:
                return None
            k = int(body["logprobs"])
        if not 0 <= k <= 20:
            raise APIError(400, "top logprobs must be between 0 and 20")
        return k

    def _sampling(self, body: dict, model: str, n_prompt: int, chat: bool = True) -> dict:
        limit = self.context_limit(model)
        if n_prompt >= limit:
            raise APIError(400, f"This model's maximum context length is {limit} tokens; the prompt has "
                                f"{n_prompt} tokens.")
        mt = body.get("max_completion_tokens", body.get("max_tokens"))
        mt = int(mt) if mt is not None else max(1, min(4096, limit - n_prompt))
        if mt <= 0:
            raise APIError(400, "max_tokens must be positive")
        mt = min(mt, limit - n_prompt)
        t = body.get("temperature")
        tp = body.get("top_p")
        if t is not None and not (0.0 <= float(t) <= 2.0):
            raise APIError(400, "temperature must be in [0, 2]")
        n = body.get("n")
        if n is not None and not (isinstance(n, int) and 1 <= n <= MAX_N):
            raise APIError(400, f"n must be an integer in [1, {MAX_N}]")
        pens = {}
        for key, lo, hi, dflt in (("frequency_penalty", -2.0, 2.0, 0.0), ("presence_penalty", -2.0, 2.0, 0.0),
                                  ("repetition_penalty", 1e-6, 10.0, 1.0)):
            v = body.get(key)
            v = dflt if v is None else float(v)
            if not lo <= v <= hi:
                raise APIError(400, f"{key} must be in [{lo:g}, {hi:g}]")
            pens[key] = v
        return {"max_tokens": mt, "temperature": 1.0 if t is None else float(t),
                "top_p": 1.0 if tp is None else float(tp), "top_k": int(body.get("top_k") or 0),
                "seed": body.get("seed"), "ignore_eos": bool(body.get("ignore_eos", False)),
                "min_tokens": int(body.get("min_tokens") or 0),
                "stop_token_ids": list(body.get("stop_token_ids") or []),
                "logprobs": self._logprobs_arg(body, chat), **pens}

    async def _run(self, endpoint: str, body: dict, prompt_ids: list, model: str, chat: bool,
                   xrid: Optional[str] = None, t_recv: Optional[float] = None):
        stream = bool(body.get("stream", False))
        rtype = "stream" if stream else "unary"
        sampling = self._sampling(body, model, len(prompt_ids), chat)
        want_lp = sampling["logprobs"] is not None
        n_choices = int(body.get("n") or 1)
        stops = body.get("stop") or []
        if isinstance(stops, str):
            stops = [stops]
        rid = ("chatcmpl-" if chat else "cmpl-") + uuid.uuid4().hex
        trace = TRACER.start(xrid or rid)
        if t_recv is not None:  # spans count from the request's arrival, before templating/tokenizing
            trace.t0 = t_recv
            trace.spans.append(("received", 0.0))
            trace.mark("tokenized")
        else:
            trace.mark("received")
        trace.attrs.update(model=model, endpoint=endpoint, prompt_tokens=len(prompt_ids), stream=stream)
        _TRACE.set(trace)
        created = int(time.time())
        tok = self.tokenizer(model)
        m = self.metrics
        m.inflight.labels(model).inc()
        m.queued.labels(model).inc()
        m.isl.labels(model).observe(len(prompt_ids))
        t0 = time.perf_counter()
        state = {"first": None, "last": {}, "n": 0, "queued": True}
        m_itl = m.itl.labels(model)

        def on_tokens(idx: int, n: int):
            """n tokens of choice idx arrived together (one worker batch)."""
            now = time.perf_counter()
            last = state["last"]
            if state["first"] is None:
                state["first"] = now
                trace.mark("first_token")
                m.ttft.labels(model).observe(now - t0)
                m.queued.labels(model).dec()
                state["queued"] = False
            elif idx in last:
                m_itl.observe(now - last[idx])
            if n > 1:  # the rest of a batch arrived with its first token: n-1 zero intervals
                _observe_zeros(m_itl, n - 1)
            last[idx] = now
            state["n"] += n

        def finish(status: str):
            m.requests.labels(model, endpoint, rtype, status).inc()
            m.inflight.labels(model).dec()
            if state["queued"]:
                m.queued.labels(model).dec()
            m.duration.labels(model).observe(time.perf_counter() - t0)
            m.osl.labels(model).observe(state["n"])
            trace.attrs.update(status=status, completion_tokens=state["n"])
            TRACER.finish(trace)

        def sub_request(idx: int) -> tuple:
            """Choice idx of an n > 1 request: its own request id and seed (same prompt, so the
            choices after the first hit the prefix cache)."""
            if n_choices == 1:
                return rid, sampling
            sp = dict(sampling)
            if sp.get("seed") is not None:
                sp["seed"] = int(sp["seed"]) + idx
            return f"{rid}-{idx}", sp

        async def events(idx: int = 0):
            """Yields (text_delta, finish_reason|None, logprob events).  With stop strings, text that
            could still be the start of a stop string is held back until it is disambiguated; the
            log-probs of the tokens behind held-back text travel with the next delta."""
            detok = IncrementalDetokenizer(tok, prompt_tail=prompt_ids[-5:])
            full, emitted = "", 0
            hold = max((len(x) for x in stops if x), default=1) - 1
            lps: list = []
            sub_rid, sub_sp = sub_request(idx)
            eos_ids = tok.eos_token_ids
            async for evs in self.generate_tokens(model, prompt_ids, sub_sp, sub_rid):
                if evs[0].timing and "worker_ms" not in trace.attrs:
                    tm = dict(evs[0].timing)  # queue / prefill / kv transfer on the worker
                    emit = tm.pop("emit_unix", None)
                    if emit is not None:  # worker emitted the first token -> this process has it
                        tm["delivery_ms"] = round((time.time() - emit) * 1e3, 3)
                    trace.attrs["worker_ms"] = tm
                on_tokens(idx, len(evs))
                ev = evs[-1]  # a batch becomes one delta; only its last event can finish the request
                eos_hit = ev.finished and ev.finish_reason == "stop" and ev.token_id in eos_ids
                body = evs[:-1] if eos_hit else evs
                full += detok.add_many([e.token_id for e in body])
                if want_lp:
                    lps.extend(e for e in body if e.logprob is not None)
                if ev.finished:
                    full += detok.flush()
                reason = ("stop" if ev.finish_reason == "abort" else ev.finish_reason) if ev.finished else None
                if stops:
                    lo = max(0, emitted - hold)
                    hits = [i for i in (full.find(x, lo) for x in stops if x) if i >= 0]
                    if hits:
                        yield full[emitted:min(hits)], "stop", lps
                        return
                    end = len(full) if ev.finished else max(emitted, len(full) - hold)
                else:
                    end = len(full)
                delta = full[emitted:end]
                emitted = end
                if delta or reason:
                    yield delta, reason, lps
                    lps = []
                if ev.finished:
                    return

        def tok_str(t: int) -> str:
            return tok.decode([int(t)], skip_special_tokens=False)

        def lp_payload(evs: list, offset: int = 0):
            """OpenAI logprobs object for these tokens (chat: content list; completions: arrays)."""
            if not want_lp:
                return None
            if chat:
                def ent(t, lp):
                    s = tok_str(t)
                    return {"token": s, "logprob": lp, "bytes": list(s.encode("utf-8", "replace"))}
                return {"content": [dict(ent(e.token_id, e.logprob),
                                         top_logprobs=[ent(t, lp) for t, lp in (e.top_logprobs or [])])
                                    for e in evs]}
            toks = [tok_str(e.token_id) for e in evs]
            offs, o = [], offset
            for s in toks:
                offs.append(o)
                o += len(s)
            return {"tokens": toks, "token_logprobs": [e.logprob for e in evs],
                    "top_logprobs": [{tok_str(t): lp for t, lp in (e.top_logprobs or [])} for e in evs],
                    "text_offset": offs}

        obj = "chat.completion" if chat else "text_completion"
        if not stream:
            async def one_choice(idx: int) -> dict:
                parts, reason, lp_evs = [], None, []
                async for d, r, evs in events(idx):
                    parts.append(d)
                    lp_evs.extend(evs)
                    reason = r or reason
                text = "".join(parts)
                if chat:
                    reasoning, text = split_text(text, self.reasoning_parser)
                    msg = {"role": "assistant", "content": text}
                    if reasoning is not None:
                        msg["reasoning_content"] = reasoning
                    choice = {"index": idx, "message": msg, "finish_reason": reason or "stop"}
                else:
                    choice = {"index": idx, "text": text, "logprobs": None, "finish_reason": reason or "stop"}
                if want_lp:
                    choice["logprobs"] = lp_payload(lp_evs)
                return choice

            try:
                choices = list(await asyncio.gather(*(one_choice(i) for i in range(n_choices))))
            except APIError:
                finish("error")
                raise
            except Exception as e:  # noqa: BLE001
                finish("error")
                raise APIError(500, f"generation failed: {e}", "server_error")
            finish("success")
            return JSONResponse({"id": rid, "object": obj, "created": created, "model": model, "choices": choices,
                                 "usage": {"prompt_tokens": len(prompt_ids), "completion_tokens": state["n"],
                                           "total_tokens": len(prompt_ids) + state["n"]}})

        include_usage = bool((body.get("stream_options") or {}).get("include_usage"))
        chunk_obj = "chat.completion.chunk" if chat else "text_completion"

        sent = [0] * n_choices  # characters streamed per choice (completions text_offset)

        splitters = ([ReasoningSplitter(self.reasoning_parser) for _ in range(n_choices)]
                     if chat and self.reasoning_parser else None)

        fast: dict = {}  # idx -> (prefix, suffix) of a plain content chunk: only the delta is encoded

        def chunk(delta: Optional[str], reason: Optional[str], first: bool = False, evs: tuple = (),
                  idx: int = 0, reasoning: Optional[str] = None) -> bytes:
            if delta and reason is None and not first and not reasoning and not want_lp:
                ps = fast.get(idx)
                if ps is None:
                    ch0 = ({"index": idx, "delta": {"content": "\x00"}, "finish_reason": None} if chat else
                           {"index": idx, "text": "\x00", "logprobs": None, "finish_reason": None})
                    t = "data: " + json.dumps({"id": rid, "object": chunk_obj, "created": created, "model": model,
                                               "choices": [ch0]}) + "\n\n"
                    ps = fast[idx] = tuple(t.split('"\\u0000"'))
                if not chat:
                    sent[idx] += len(delta)
                return (ps[0] + json.dumps(delta) + ps[1]).encode()
            if chat:
                d = {}
                if first:
                    d["role"] = "assistant"
                if reasoning:
                    d["reasoning_content"] = reasoning
                if delta is not None:
                    d["content"] = delta
                ch = {"index": idx, "delta": d, "finish_reason": reason}
                if want_lp and not first:
                    ch["logprobs"] = lp_payload(list(evs))
            else:
                ch = {"index": idx, "text": delta or "", "logprobs": lp_payload(list(evs), sent[idx]),
                      "finish_reason": reason}
                sent[idx] += len(delta or "")
            return ("data: " + json.dumps({"id": rid, "object": chunk_obj, "created": created, "model": model,
                                           "choices": [ch]}) + "\n\n").encode()

        async def sse():
            status = "success"
            try:
                if chat:
                    for i in range(n_choices):
                        yield chunk("", None, first=True, idx=i)
                async for i, (d, r, evs) in _merge([events(i) for i in range(n_choices)]):
                    rd = None
                    if splitters is not None:
                        rd, d = splitters[i].feed(d, final=bool(r))
                    if d or r or rd:
                        yield chunk(d if d else ("" if r else None), r, evs=evs, idx=i, reasoning=rd)
                if include_usage:
                    yield ("data: " + json.dumps({"id": rid, "object": chunk_obj, "created": created, "model": model,
                                                  "choices": [], "usage": {"prompt_tokens": len(prompt_ids),
                                                                           "completion_tokens": state["n"],
                                                                           "total_tokens": len(prompt_ids) + state["n"]}})
                           + "\n\n").encode()
                yield b"data: [DONE]\n\n"
            except APIError as e:
                status = "error"
                yield ("data: " + json.dumps({"error": {"message": e.message, "type": e.etype, "code": e.status}})
                       + "\n\n").encode()
            except Exception as e:  # noqa: BLE001
                status = "error"
                yield ("data: " + json.dumps({"error": {"message": str(e), "type": "server_error"}}) + "\n\n").encode()
            finally:
                finish(status)

        return StreamingResponse(sse(), media_type="text/event-stream",
                                 headers={"Cache-Control": "no-cache", "X-Request-Id": xrid or rid})

    # ---------------------------------------------------------------- app
    def _build_app(self) -> FastAPI:
        app = FastAPI(title="mxserve frontend", lifespan=self._lifespan)
        fe = self

        @app.exception_handler(APIError)
        async def _api_err(_req, e: APIError):
            return _err(e.status, e.message, e.etype)

        @app.get("/v1/models")
        async def models():
            data = [{"id": m, "object": "model", "created": int(fe.started), "owned_by": "mxserve"}
                    for m in fe.registry.models()]
            return {"object": "list", "data": data}

        @app.post("/v1/chat/completions")
        async def chat(request: HTTPRequest):
            try:
                body = await request.json()
            except Exception:  # noqa: BLE001
                return _err(400, "invalid JSON body")
            if not isinstance(body, dict) or "messages" not in body:
                return _err(400, "`messages` is required")
            t_recv = time.perf_counter()
            model = fe.resolve_model(body.get("model"))
            try:
                cfg = fe.model_cfg(model)
                text = render(cfg.chat_template, body["messages"], find_local_model_dir(cfg.name))
            except ValueError as e:
                return _err(400, str(e))
            ids = fe.tokenizer(model).encode(text)
            return await fe._run("chat_completions", body, ids, model, chat=True,
                                 xrid=request.headers.get("x-request-id"), t_recv=t_recv)

        @app.post("/v1/completions")
        async def completions(request: HTTPRequest):
            try:
                body = await request.json()
            except Exception:  # noqa: BLE001
                return _err(400, "invalid JSON body")
            t_recv = time.perf_counter()
            model = fe.resolve_model(body.get("model"))
            p = body.get("prompt")
            if isinstance(p, list) and p and isinstance(p[0], int):
                ids = list(p)
            elif isinstance(p, str):
                ids = fe.tokenizer(model).encode(p, add_special_tokens=True)
            else:
                return _err(400, "`prompt` must be a string or a list of token ids")
            return await fe._run("completions", body, ids, model, chat=False,
                                 xrid=request.headers.get("x-request-id"), t_recv=t_recv)

        @app.get("/debug/traces")
        async def traces(n: int = 100):
            return {"traces": TRACER.recent(n)}

        @app.get("/health")
        async def health():
            ws = fe.registry.list()
            if not ws:
                return JSONResponse({"status": "no workers", "workers": []}, status_code=503)
            return {"status": "healthy", "models": fe.registry.models(), "workers": len(ws)}

        @app.get("/live")
        async def live():
            return {"status": "alive"}

        @app.get("/metrics")
        async def metrics():
            for role in ("agg", "prefill", "decode"):
                for model in fe.registry.models():
                    fe.metrics.workers.labels(model, role).set(len(fe.registry.list(model, role)))
            return Response(fe.metrics.render(), media_type="text/plain; version=0.0.4")

        @app.post("/internal/register")
        async def register(request: HTTPRequest):
            d = await request.json()
            info = fe.apply_register(d)
            if fe.bus is not None:  # the sibling processes of a multi-process frontend
                fe.bus.publish("register", d)
            return {"ok": True, "index": info.index}

        @app.post("/internal/heartbeat")
        async def heartbeat(request: HTTPRequest):
            d = await request.json()
            ok = fe.apply_heartbeat(d)
            if fe.bus is not None:
                fe.bus.publish("heartbeat", d)
            return JSONResponse({"ok": ok}, status_code=200 if ok else 404)

        @app.get("/internal/workers")
        async def workers():
            return {"workers": [w.public() for w in fe.registry.list()]}

        return app

    @contextlib.asynccontextmanager
    async def _lifespan(self, app):
        async def reaper():
            while True:
                await asyncio.sleep(1.0)
                for wid in self.registry.expire():
                    log.warning("worker %s lease expired", wid)
        task = asyncio.get_running_loop().create_task(reaper())
        if self.bus is not None:
            self.bus.start(asyncio.get_running_loop(), self.apply_peer)
        yield
        task.cancel()
        for mc in self._mux.values():
            mc.reset()
        if self._http is not None:
            await self._http.close()
            self._http = None


def serve_app(fe: Frontend, host: str = "0.0.0.0", port: int = 8000, sock=None) -> None:
    """Serve a Frontend until SIGTERM / SIGINT: our HTTP/1.1 server with the push-streaming fast
    path (httpd.py + fastpath.py; the default), or uvicorn (MXS_FRONTEND_SERVER=uvicorn)."""
    from ..utils.gcpause import freeze_heap
    freeze_heap()  # no full collections over the start-up heap while streaming (utils/gcpause.py)
    if os.environ.get("MXS_FRONTEND_SERVER", "httpd") == "uvicorn":
        import uvicorn
        if sock is not None:
            uvicorn.Server(uvicorn.Config(fe.app, log_level="warning", access_log=False)).run(sockets=[sock])
        else:
            uvicorn.run(fe.app, host=host, port=port, log_level="warning", access_log=False)
        return
    from . import fastpath, httpd

    def fast(req, conn):
        return fastpath.handle(fe, req, conn)
    prof = os.environ.get("MXS_FRONTEND_PROFILE")  # dev: cProfile of this process -> <path>.<pid>
    if prof:
        import cProfile
        cProfile.runctx("run(app, host, port, fast=fast, sock=sock)", {},
                        {"run": httpd.run, "app": fe.app, "host": host, "port": port, "fast": fast, "sock": sock},
                        f"{prof}.{os.getpid()}")
        return
    httpd.run(fe.app, host, port, fast=fast, sock=sock)
