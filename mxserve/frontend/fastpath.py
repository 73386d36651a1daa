"""Push-based SSE streaming: the frontend's hot path under its own HTTP server (httpd.py).

A streamed chat / completion request with one choice, no log-probs and no reasoning parser -- what
chat.sh, multi_convos_parallel.sh and the benchmark clients send -- is served here.  Its tokens are
pushed, on the event-loop thread, from the worker channel's reader (MuxClient._read demultiplexes a
worker line per engine step) straight into the client's connection: detokenize, stop strings, one
SSE chunk, transport.write.  No per-token task switch, no generator chain, no ASGI/h11 layers; the
request's own coroutine only routes, waits for the end, retries before the first token and migrates
a broken stream (same policy as Frontend.generate_tokens).  Every other request (unary, n > 1,
logprobs, ...) goes to the FastAPI routes, which produce identical bytes for what both serve.
"""
from __future__ import annotations

import asyncio
import bisect
import json
import logging
import time
import uuid
from typing import Optional

from ..utils.tracing import TRACER
from .chat_template import render
from .tokenizer import IncrementalDetokenizer

# a client that reads slower than this much buffered output is dropped (its request is aborted)
MAX_BUFFERED = 16 << 20


log = logging.getLogger("mxserve.frontend.fastpath")


class ClientGone(ConnectionError):
    pass


class _LocalHistogram:
    """One request's share of a prometheus Histogram child, counted locally (a list index per
    observation) and added to the shared child every FLUSH observations and at the end: the
    multiprocess-mode child takes a lock and an mmap write per inc()."""
    FLUSH = 64

    def __init__(self, child):
        self.child = child
        self.ub = child._upper_bounds
        self.counts = [0] * len(self.ub)
        self.sum = 0.0
        self.n = 0

    def observe(self, v: float) -> None:
        i = bisect.bisect_left(self.ub, v)
        self.counts[i if i < len(self.ub) else -1] += 1
        self.sum += v
        self.n += 1
        if self.n >= self.FLUSH:
            self.flush()

    def flush(self) -> None:
        if not self.n:
            return
        b = self.child._buckets
        for i, c in enumerate(self.counts):
            if c:
                b[i].inc(c)
                self.counts[i] = 0
        self.child._sum.inc(self.sum)
        self.sum, self.n = 0.0, 0


class PushStream:
    """One streamed choice: token events -> SSE bytes on the connection, plus the frontend metrics
    the FastAPI path records (TTFT, ITL, ISL / OSL, request counts, duration)."""

    def __init__(self, fe, conn, model: str, chat: bool, body: dict, prompt_ids: list, sampling: dict,
                 xrid: Optional[str], t_recv: float):
        self.fe, self.conn, self.model, self.chat = fe, conn, model, chat
        self.prompt_ids = prompt_ids
        self.sampling = sampling
        self.rid = ("chatcmpl-" if chat else "cmpl-") + uuid.uuid4().hex
        self.xrid = xrid
        self.created = int(time.time())
        tok = fe.tokenizer(model)
        self.eos_ids = tok.eos_token_ids
        self.detok = IncrementalDetokenizer(tok, prompt_tail=prompt_ids[-5:])
        stops = body.get("stop") or []
        self.stops = [stops] if isinstance(stops, str) else [x for x in stops if x]
        self.hold = max((len(x) for x in self.stops), default=1) - 1
        self.include_usage = bool((body.get("stream_options") or {}).get("include_usage"))
        self.full, self.emitted, self.sent = "", 0, 0
        self.generated: list = []  # token ids so far (migration re-prefills prompt + these)
        self.done = False  # the response's last choice chunk is written
        self.worker_done = False  # the worker ended the request itself (no abort needed)
        self.obj = "chat.completion.chunk" if chat else "text_completion"
        ch0 = ({"index": 0, "delta": {"content": "\x00"}, "finish_reason": None} if chat else
               {"index": 0, "text": "\x00", "logprobs": None, "finish_reason": None})
        t = "data: " + json.dumps({"id": self.rid, "object": self.obj, "created": self.created, "model": model,
                                   "choices": [ch0]}) + "\n\n"
        self.pre, self.post = t.split('"\\u0000"')
        m = fe.metrics
        self.m_itl = m.itl.labels(model)
        self.itl = _LocalHistogram(self.m_itl)
        self.first = None
        self.last = None
        self.n = 0
        self.t0 = time.perf_counter()
        self.trace = TRACER.start(xrid or self.rid)
        self.trace.t0 = t_recv
        self.trace.spans.append(("received", 0.0))
        self.trace.mark("tokenized")
        self.trace.attrs.update(model=model, endpoint="chat_completions" if chat else "completions",
                                prompt_tokens=len(prompt_ids), stream=True)
        m.inflight.labels(model).inc()
        m.queued.labels(model).inc()
        m.isl.labels(model).observe(len(prompt_ids))

    # ------------------------------------------------------------------ bytes
    def _chunk(self, choice: dict) -> bytes:
        return ("data: " + json.dumps({"id": self.rid, "object": self.obj, "created": self.created,
                                       "model": self.model, "choices": [choice]}) + "\n\n").encode()

    def head(self) -> None:
        c = self.conn
        c.write_head(200, [(b"content-type", b"text/event-stream; charset=utf-8"), (b"cache-control", b"no-cache"),
                           (b"x-request-id", (self.xrid or self.rid).encode()), (b"transfer-encoding", b"chunked")])
        if self.chat:
            c.write_chunk(self._chunk({"index": 0, "delta": {"role": "assistant", "content": ""},
                                       "finish_reason": None}))

    def _emit(self, delta: str, reason: Optional[str]) -> None:
        if reason is None:
            if delta:
                self.conn.write_chunk((self.pre + json.dumps(delta) + self.post).encode())
            return
        if self.chat:
            data = self._chunk({"index": 0, "delta": {"content": delta}, "finish_reason": reason})
        else:
            data = self._chunk({"index": 0, "text": delta, "logprobs": None, "finish_reason": reason})
        self.conn.write_chunk(data)
        self.done = True

    # ------------------------------------------------------------------ tokens (event-loop thread)
    def on_events(self, evs: list) -> bool:
        """TokenEvents of this request (the pulled /generate path): see _tokens."""
        ev = evs[-1]
        return self._tokens([e.token_id for e in evs], ev.finished, ev.finish_reason, evs[0].timing)

    def on_payload(self, d: dict) -> bool:
        """One worker line's entry for this request (mux channel: {"t": id | [ids], "f", "r", ...},
        worker/server.py _batch_dict) straight from the channel reader, no TokenEvent objects."""
        toks = d["t"]
        if not isinstance(toks, list):
            toks = [toks]
        for i, t in enumerate(toks):
            if t < 0:
                if i:  # the tokens before the marker were generated: deliver them (they count for migration)
                    self._tokens(toks[:i], False, None, d.get("tm"))
                if t == -2:  # the worker dropped the stream (fault injection): retry / migrate
                    raise ConnectionError("worker dropped the stream")
                raise RuntimeError("worker failed the request")
        return self._tokens(toks, d["f"], d["r"], d.get("tm"))

    def _tokens(self, toks: list, fin: bool, finish_reason: Optional[str], timing: Optional[dict]) -> bool:
        """Write what these tokens add to the text; True once the response has its final choice."""
        if self.conn.closed:
            raise ClientGone("client disconnected")
        if self.conn.buffered() > MAX_BUFFERED:
            raise ClientGone("client is not reading its stream")
        now = time.perf_counter()
        k = len(toks)
        if self.first is None:
            self.first = now
            self.trace.mark("first_token")
            m = self.fe.metrics
            m.ttft.labels(self.model).observe(now - self.t0)
            m.queued.labels(self.model).dec()
            if timing and "worker_ms" not in self.trace.attrs:
                tm = dict(timing)
                emit = tm.pop("emit_unix", None)
                if emit is not None:
                    tm["delivery_ms"] = round((time.time() - emit) * 1e3, 3)
                self.trace.attrs["worker_ms"] = tm
        elif self.last is not None:
            self.itl.observe(now - self.last)
        if k > 1:  # the rest of a batch arrived with its first token: k - 1 zero intervals
            self.itl.counts[0] += k - 1
            self.itl.n += k - 1
        self.last = now
        self.n += k
        self.generated.extend(toks)
        if fin:
            self.worker_done = True
            if finish_reason == "stop" and toks[-1] in self.eos_ids:
                toks = toks[:-1]
        if len(toks) == 1:
            text = self.detok.add(toks[0])
        else:
            text = self.detok.add_many(toks) if toks else ""
        if fin:
            text += self.detok.flush()
        reason = ("stop" if finish_reason == "abort" else finish_reason) if fin else None
        if not self.stops:  # the common case: no text is held back, nothing accumulates
            if text or reason:
                self._emit(text, reason)
            return fin
        self.full += text
        lo = max(0, self.emitted - self.hold)
        hits = [i for i in (self.full.find(x, lo) for x in self.stops) if i >= 0]
        if hits:
            self._emit(self.full[self.emitted:min(hits)], "stop")
            return True
        end = len(self.full) if fin else max(self.emitted, len(self.full) - self.hold)
        delta = self.full[self.emitted:end]
        self.emitted = end
        if delta or reason:
            self._emit(delta, reason)
        return fin

    # ------------------------------------------------------------------ end
    def finish_ok(self) -> None:
        c = self.conn
        if self.include_usage:
            np_ = len(self.prompt_ids)
            c.write_chunk(("data: " + json.dumps({"id": self.rid, "object": self.obj, "created": self.created,
                                                  "model": self.model, "choices": [],
                                                  "usage": {"prompt_tokens": np_, "completion_tokens": self.n,
                                                            "total_tokens": np_ + self.n}}) + "\n\n").encode())
        c.write_chunk(b"data: [DONE]\n\n")

    def finish_error(self, message: str, etype: str = "server_error", code: Optional[int] = None) -> None:
        err = {"message": message, "type": etype}
        if code is not None:
            err["code"] = code
        self.conn.write_chunk(("data: " + json.dumps({"error": err}) + "\n\n").encode())

    def record(self, status: str, endpoint: str) -> None:
        self.itl.flush()
        m = self.fe.metrics
        m.requests.labels(self.model, endpoint, "stream", status).inc()
        m.inflight.labels(self.model).dec()
        if self.first is None:
            m.queued.labels(self.model).dec()
        m.duration.labels(self.model).observe(time.perf_counter() - self.t0)
        m.osl.labels(self.model).observe(self.n)
        self.trace.attrs.update(status=status, completion_tokens=self.n)
        TRACER.finish(self.trace)


def eligible(fe, path: str, body) -> bool:
    """Requests the push path serves; the rest keep the FastAPI routes."""
    if not isinstance(body, dict) or not body.get("stream"):
        return False
    if (body.get("n") or 1) != 1 or fe.local:
        return False
    chat = path == "/v1/chat/completions"
    if chat and (body.get("logprobs") or body.get("top_logprobs") is not None or fe.reasoning_parser):
        return False
    if not chat and body.get("logprobs") is not None:
        return False
    return True


async def handle(fe, req, conn) -> bool:
    """httpd fast hook: True if the request was served here."""
    if req.method != "POST" or req.path not in ("/v1/chat/completions", "/v1/completions"):
        return False
    try:
        body = json.loads(req.body)
    except ValueError:
        return False  # the FastAPI route answers malformed bodies
    if not eligible(fe, req.path, body):
        return False
    from .app import APIError
    chat = req.path == "/v1/chat/completions"
    t_recv = time.perf_counter()
    try:
        model = fe.resolve_model(body.get("model"))
        if chat:
            if "messages" not in body:
                raise APIError(400, "`messages` is required")
            cfg = fe.model_cfg(model)
            from ..models.config import find_local_model_dir
            try:
                text = render(cfg.chat_template, body["messages"], find_local_model_dir(cfg.name))
            except ValueError as e:
                raise APIError(400, str(e))
            ids = fe.tokenizer(model).encode(text)
        else:
            p = body.get("prompt")
            if isinstance(p, list) and p and isinstance(p[0], int):
                ids = list(p)
            elif isinstance(p, str):
                ids = fe.tokenizer(model).encode(p, add_special_tokens=True)
            else:
                raise APIError(400, "`prompt` must be a string or a list of token ids")
        sampling = fe._sampling(body, model, len(ids), chat)
    except APIError as e:
        data = json.dumps({"error": {"message": e.message, "type": e.etype, "code": e.status}}).encode()
        conn.write_head(e.status, [(b"content-type", b"application/json"), (b"content-length", str(len(data)).encode())])
        conn.write(data)
        conn.finish()
        return True
    xrid = req.header(b"x-request-id")
    ps = PushStream(fe, conn, model, chat, body, ids, sampling, xrid.decode() if xrid else None, t_recv)
    endpoint = "chat_completions" if chat else "completions"
    task = asyncio.current_task()
    conn.on_close.append(task.cancel)  # the client left: stop routing / waiting, abort on the worker
    status, reason, err = "success", "ok", None
    ps.head()
    try:
        await fe.run_push(model, ids, sampling, ps.rid, ps)
        ps.finish_ok()
    except asyncio.CancelledError:
        status, reason = "error", "client_gone"
    except APIError as e:
        status, reason, err = "error", f"api_error_{e.status}", e
        ps.finish_error(e.message, e.etype, e.status)
    except Exception as e:  # noqa: BLE001 - reported in the stream, like the FastAPI path
        status, reason, err = "error", f"error_{type(e).__name__}", e
        ps.finish_error(str(e))
    finally:
        ps.record(status, endpoint)
        fe.metrics.stream_close.labels(model, reason).inc()
        if reason != "ok":
            log.warning("stream %s closed early: %s after %d tokens%s", ps.rid, reason, ps.n,
                        f" ({err!r})" if err is not None else "")
        conn.end_chunked()
        conn.finish()
    return True
